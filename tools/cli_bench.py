"""End-to-end CLI frames/s at 1080p on one GPU: the reference's frame-directory
path (pipeline.py --input_dir: PIL decode -> stylize -> LAB EMA -> blend -> PIL encode, pipeline.py:1080-2119) through
this engine's pipeline.main, for PNG and JPEG frames, beside the host decode / encode rates alone (the same thread
count) and the GPU step rate -- so the host I/O share of the wall time is measured, not assumed.

  python tools/cli_bench.py [--frames 48] [--threads 16]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch
from PIL import Image

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=48)
    ap.add_argument("--threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "16") or 16))
    args = ap.parse_args()
    from neuralstyletransferv1_amd import pipeline as P
    from neuralstyletransferv1_amd import synthetic

    tmp = tempfile.mkdtemp(prefix="nst_cli_")
    ck = os.path.join(tmp, "johnson.pth")
    torch.save(synthetic.make_state_dict("johnson", 0), ck)
    frames = synthetic.make_frames(8, 1080, 1920, seed=300)
    res = {"frames": args.frames, "threads": args.threads, "frame_hw": [1080, 1920]}
    pool = ThreadPoolExecutor(args.threads)
    for ext in ("png", "jpg"):
        d_in = os.path.join(tmp, f"in_{ext}")
        os.makedirs(d_in)
        paths = [os.path.join(d_in, f"frame_{i + 1:04d}.{ext}") for i in range(args.frames)]

        def enc(i):
            im = Image.fromarray(frames[i % len(frames)])
            if ext == "png":
                im.save(paths[i])
            else:
                im.save(paths[i], format="JPEG", quality=85)
        t0 = time.perf_counter()
        list(pool.map(enc, range(args.frames)))
        t_enc = time.perf_counter() - t0
        t0 = time.perf_counter()
        list(pool.map(lambda p: np.asarray(Image.open(p).convert("RGB")), paths))
        t_dec = time.perf_counter() - t0
        d_out = os.path.join(tmp, f"out_{ext}")
        argv = ["--input_dir", d_in, "--output_dir", d_out, "--model", ck, "--io_preset", "imagenet_255",
                "--dtype", "bf16", "--batch", "8", "--blend", "0.9", "--smooth_alpha", "0.65", "--image_ext", ext,
                "--threads", str(args.threads), "--work_dir", os.path.join(tmp, f"w_{ext}")]
        P.main(argv[:4] + ["--max_frames", "8"] + argv[4:])  # warm-up: model load, kernels, LAB tables
        t0 = time.perf_counter()
        rc = P.main(argv)
        t_cli = time.perf_counter() - t0
        assert rc == 0
        res[ext] = {"cli_frames_per_s": round(args.frames / t_cli, 2), "cli_s": round(t_cli, 3),
                    "host_encode_frames_per_s": round(args.frames / t_enc, 2),
                    "host_decode_frames_per_s": round(args.frames / t_dec, 2)}
        print(ext, json.dumps(res[ext]), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
