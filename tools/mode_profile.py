"""Per-layer kernel times (HIP events on the forward's stream) of the Johnson 1080p batch-8 step in one
compute dtype, plus the step's frames/s: python tools/mode_profile.py [fp32s|fp32|bf16|fp16] [arch].  Prints one
JSON line.  Used for tile sweeps of the generic kernels (NST_HIP_LIB selects a library build)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neuralstyletransferv1_amd import synthetic  # noqa: E402

dt = sys.argv[1] if len(sys.argv) > 1 else "fp32s"
arch = sys.argv[2] if len(sys.argv) > 2 else "johnson"
dev = torch.device("cuda", 0)
frames = torch.from_numpy(synthetic.make_frames(8, 1080, 1920, seed=5)).to(dev)
m = synthetic.build_module(arch)
m.load_state_dict(synthetic.make_state_dict(arch, 0))
m = m.to(dev).eval()
m.compute_dtype = dt
m.kernel_select = frozenset(k for k in os.environ.get("MODE_KSEL", "").split(",") if k)  # e.g. no_wstat,no_ws2
eng = m.engine(dev)
for _ in range(2):
    eng.stylize_u8(frames, "imagenet_255")
torch.cuda.synchronize()
t0 = time.perf_counter()
K = 5
for _ in range(K):
    eng.stylize_u8(frames, "imagenet_255")
torch.cuda.synchronize()
step = (time.perf_counter() - t0) / K
eng.profile_begin()
for _ in range(3):
    eng.stylize_u8(frames, "imagenet_255")
torch.cuda.synchronize()
prof = eng.profile_end()
print(json.dumps({"arch": arch, "dtype": dt, "lib": os.environ.get("NST_HIP_LIB", "default"),
                  "ksel": sorted(m.kernel_select), "frames_per_s": round(8 / step, 1),
                  "ms_per_step": round(step * 1e3, 3),
                  "per_layer_ms": {n: round(ms / max(c, 1), 3) for n, ms, c in prof}}), flush=True)
