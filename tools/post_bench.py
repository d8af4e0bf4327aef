"""Throughput of the non-conv hot-path kernels (scratch measurement, numbers quoted in DESIGN.md):
  * lab_ema_kernel (pipeline.py:1942-1978 LAB L-EMA through the LittleCMS tables) on 8 frames of
    1080p and 4K: frames/s and GB/s of algorithmic bytes (3 B in + 3 B out + 4 B state read + 4 B
    state write per pixel; the two table gathers are not counted);
  * nst_gram (utils.py:80-83) at the VGG-19 style layers of a 512x512 image, bf16 HWC: us and TFLOP/s.
  * the temporal stage at 1080p: Farneback flow, the flow-fused EMA, the motion alpha.
HIP events on the current stream."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neuralstyletransferv1_amd import _lib, synthetic  # noqa: E402
from neuralstyletransferv1_amd.postproc import LabSmoother  # noqa: E402
from neuralstyletransferv1_amd.utils import gram_raw  # noqa: E402

dev = torch.device("cuda", 0)


def timed(fn, k=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(k):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / k


for (h, w) in ((1080, 1920), (2160, 3840)):
    fr = torch.from_numpy(synthetic.make_frames(8, h, w, seed=3)).to(dev)
    sm = LabSmoother(dev, True, 0.65)
    out = torch.empty_like(fr)
    ms = timed(lambda: sm(fr, out))
    px = 8 * h * w
    print(f"lab_ema {w}x{h} x8: {ms:.3f} ms  {8 / ms * 1e3:.0f} frames/s  {px * 14 / ms / 1e6:.0f} GB/s algorithmic",
          flush=True)

for c, hw in ((64, 512 * 512), (128, 256 * 256), (256, 128 * 128), (512, 64 * 64), (512, 32 * 32)):
    x = torch.relu(torch.randn(1, hw, c, device=dev)).to(torch.bfloat16)
    ms = timed(lambda: gram_raw(x, _lib.NST_DT_BF16, _lib.NST_GRAM_HWC, 1, c, hw))
    print(f"gram c={c} hw={hw}: {ms * 1e3:.1f} us  {2 * c * c * hw / ms / 1e9:.1f} TFLOP/s  "
          f"{hw * c * 2 / ms / 1e6:.0f} GB/s of F", flush=True)

# temporal stage (--flow_ema --flow_method farneback, --motion_blend): one 1080p frame pair
from neuralstyletransferv1_amd import temporal as T  # noqa: E402

fr = torch.from_numpy(synthetic.make_frames(2, 1080, 1920, seed=5)).to(dev)
g = T.gray_u8(fr)
sc = T.FlowScratch()
ms = timed(lambda: T.farneback(g[0], g[1], sc), 10)
print(f"farneback 1920x1080 (0.5, 3 levels, 15, 3 iterations, 5, 1.1): {ms:.3f} ms per frame", flush=True)
fl = T.farneback(g[0], g[1], sc)
o1 = torch.rand(3, 1080, 1920, device=dev)
o0 = torch.rand(3, 1080, 1920, device=dev)
ms = timed(lambda: T.fuse(o1, o0, fl, 0.85))
print(f"flow fuse 1920x1080: {ms * 1e3:.1f} us  {1080 * 1920 * (12 * 3 + 8) / ms / 1e6:.0f} GB/s algorithmic", flush=True)
ms = timed(lambda: T.motion_alpha(fl, 0.9))
print(f"motion alpha 1920x1080: {ms * 1e3:.1f} us", flush=True)
