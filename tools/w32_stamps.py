"""Cycle breakdown of the trunk kernel (conv_wst16.hip, or conv_wst32.hip) from its s_memtime intervals (diagnostic library: `make stamp`,
then NST_HIP_LIB=.../libnst_hip_stamp.so python tools/w32_stamps.py).  The last trunk launch of the step
(res5.conv2, a plain conv) leaves the sums per wave.  Scratch measurement."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neuralstyletransferv1_amd import _lib, synthetic  # noqa: E402
from neuralstyletransferv1_amd.transformer_net import TransformerNet  # noqa: E402

dev = torch.device("cuda", 0)
net = TransformerNet()
net.load_state_dict(synthetic.make_state_dict("johnson", 0))
net = net.to(dev).eval()
net.compute_dtype = "bf16"
eng = net.engine(dev)
frames = torch.from_numpy(synthetic.make_frames(8, 1080, 1920, seed=5)).to(dev)
for _ in range(3):
    eng.stylize_u8(frames, "imagenet_255")
torch.cuda.synchronize()
PT = 16
n = 256 * 4 * PT
buf = (ctypes.c_longlong * n)()
L = _lib.lib()
fn = getattr(L, "nst_debug_w16_stamps", None) or getattr(L, "nst_debug_w32_stamps")
got = fn(buf, n)
a = np.frombuffer(buf, dtype=np.int64).reshape(256 * 4, PT).astype(np.float64)
tiles = a[:, 6]
ok = tiles > 0
per = a[ok, :6] / tiles[ok, None]
names = ["part0", "part1", "part2", "part3", "epilogue", "head"]
print(f"waves {ok.sum()}  tiles/wave {tiles[ok].mean():.2f}  cycles per tile (mean over waves, p10..p90):")
for k, nm in enumerate(names):
    v = per[:, k]
    print(f"  {nm:9s} {v.mean():8.0f}   ({np.percentile(v, 10):.0f} .. {np.percentile(v, 90):.0f})")
print(f"  total     {per[:, :6].sum(axis=1).mean():8.0f}")
