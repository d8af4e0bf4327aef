"""Sustained load for tools/power_probe.sh: the configs[1] batch (8 x 1080p) back to back for SECONDS seconds, then
the frames/s of the whole run.   python tools/power_load.py [seconds] [arch] [dtype]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neuralstyletransferv1_amd import synthetic  # noqa: E402

secs = float(sys.argv[1]) if len(sys.argv) > 1 else 45.0
arch = sys.argv[2] if len(sys.argv) > 2 else "johnson"
dtype = sys.argv[3] if len(sys.argv) > 3 else "bf16"
dev = torch.device("cuda", 0)
net = synthetic.build_module(arch)
net.load_state_dict(synthetic.make_state_dict(arch, 0))
net = net.to(dev).eval()
net.compute_dtype = dtype
eng = net.engine(dev)
frames = torch.from_numpy(synthetic.make_frames(8, 1080, 1920, seed=5)).to(dev)
for _ in range(3):
    eng.stylize_u8(frames, "imagenet_255")
torch.cuda.synchronize()
print("load start", flush=True)
t0 = time.perf_counter()
n = 0
while time.perf_counter() - t0 < secs:
    for _ in range(20):
        eng.stylize_u8(frames, "imagenet_255")
    torch.cuda.synchronize()
    n += 20
dt = time.perf_counter() - t0
print(f"load done: {arch} {dtype} {n * 8 / dt:.1f} frames/s over {dt:.1f} s", flush=True)
