"""GPU PNG encoder rate and file size at 1080p (csrc/png_enc.hip): one call over a batch of 8 synthetic frames and
over 8 stylized frames, HIP events on the encoder's stream; beside it the host writers (pngio Z_RLE, Pillow
default) on the same frames at --threads.  Prints one JSON line.   python tools/png_bench.py [--threads 16]"""
import argparse
import io
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    from PIL import Image

    from neuralstyletransferv1_amd import pngio, synthetic
    from neuralstyletransferv1_amd.transformer_net import TransformerNet
    dev = torch.device("cuda", 0)
    net = TransformerNet()
    net.load_state_dict(synthetic.make_state_dict("johnson", 0))
    net = net.to(dev).eval()
    net.compute_dtype = "bf16"
    eng = net.engine(dev)
    src = torch.from_numpy(synthetic.make_frames(8, 1080, 1920, seed=300)).to(dev)
    res = {"frame_hw": [1080, 1920], "batch": 8}
    pool = ThreadPoolExecutor(args.threads)
    for name, x in (("synthetic", src), ("stylized", eng.stylize_u8(src, "imagenet_255"))):
        files, sizes = pngio.encode_png_gpu(x)
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(args.reps):
            pngio.encode_png_gpu(x)
        ev1.record()
        torch.cuda.synchronize()
        ms = ev0.elapsed_time(ev1) / args.reps
        raw = 1080 * (1920 * 3 + 1)
        sz = sizes.cpu().numpy()
        host = x.cpu().numpy()
        t0 = time.perf_counter()
        rle = list(pool.map(lambda f: len(pngio.encode_png(f)), host))
        t_rle = time.perf_counter() - t0

        def pil(f):
            b = io.BytesIO()
            Image.fromarray(f).save(b, format="PNG")
            return b.tell()
        t0 = time.perf_counter()
        pl = list(pool.map(pil, host[:4]))
        t_pil = time.perf_counter() - t0
        res[name] = {"gpu_ms_per_batch": round(ms, 3), "gpu_frames_per_s": round(8 / ms * 1e3, 1),
                     "gpu_size_over_raw": round(float(sz.mean()) / raw, 4),
                     "host_zrle_frames_per_s": round(8 / t_rle, 1), "host_zrle_size_over_raw": round(np.mean(rle) / raw, 4),
                     "host_pil_frames_per_s": round(4 / t_pil, 1), "host_pil_size_over_raw": round(np.mean(pl) / raw, 4)}
        print(name, json.dumps(res[name]), flush=True)
    res["threads"] = args.threads
    print(json.dumps(res))


if __name__ == "__main__":
    main()
