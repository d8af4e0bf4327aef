"""Is the step faster as sequential sub-batches (layer outputs small enough for the 256 MB Infinity Cache)?
Times the bench's 8 1080p frames as 8/b graph-captured stylize_u8 calls of b frames, b in 1, 2, 4, 8, alternating.
python tools/batch_split_probe.py"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from neuralstyletransferv1_amd import synthetic
    from neuralstyletransferv1_amd.engine import capture_u8
    from neuralstyletransferv1_amd.transformer_net import TransformerNet
    dev = torch.device("cuda", 0)
    net = TransformerNet()
    net.load_state_dict(synthetic.make_state_dict("johnson", 0))
    net = net.to(dev).eval()
    net.compute_dtype = "bf16"
    eng = net.engine(dev)
    frames = torch.from_numpy(synthetic.make_frames(8, 1080, 1920, seed=1000)).to(dev)
    ref = eng.stylize_u8(frames, "imagenet_255").clone()
    runs = {}
    for b in (8, 4, 2, 1):
        parts = [capture_u8(eng, frames[i:i + b].contiguous(), "imagenet_255") for i in range(0, 8, b)]
        ok = all(torch.equal(o, ref[i * b:(i + 1) * b]) for i, (r, o) in enumerate(parts) if (r() or True))
        runs[b] = (parts, ok)
    res = {b: [] for b in runs}
    for rep in range(3):
        for b, (parts, ok) in runs.items():
            for _ in range(5):
                for r, _o in parts:
                    r()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(30):
                for r, _o in parts:
                    r()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / 30 * 1e3
            res[b].append(round(ms, 4))
            print(f"batch {b} x {8 // b}: {ms:.4f} ms per 8 frames ({8e3 / ms:.1f} frames/s) outputs equal {ok}", flush=True)
    print(json.dumps({str(b): v for b, v in res.items()}))


if __name__ == "__main__":
    main()
