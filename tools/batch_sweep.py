"""Per-frame time of the bf16 Johnson path at 1080p vs frames per nst_forward call (scratch measurement).
Frames per call change the per-launch working set (Infinity Cache residency) and the tile counts."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neuralstyletransferv1_amd import synthetic  # noqa: E402
from neuralstyletransferv1_amd.transformer_net import TransformerNet  # noqa: E402

dev = torch.device("cuda", 0)
net = TransformerNet()
net.load_state_dict(synthetic.make_state_dict("johnson", 0))
net = net.to(dev).eval()
net.compute_dtype = "bf16"
eng = net.engine(dev)
frames = torch.from_numpy(synthetic.make_frames(8, 1080, 1920, seed=5)).to(dev)
for nb in [int(v) for v in (sys.argv[1:] or ["8", "4", "2", "1"])]:
    chunks = [frames[i:i + nb].contiguous() for i in range(0, 8, nb)]
    for _ in range(3):
        for c in chunks:
            eng.stylize_u8(c, "imagenet_255")
    torch.cuda.synchronize()
    t = time.perf_counter()
    K = 10
    for _ in range(K):
        for c in chunks:
            eng.stylize_u8(c, "imagenet_255")
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / K
    eng.profile_begin()
    for _ in range(3):
        for c in chunks:
            eng.stylize_u8(c, "imagenet_255")
    torch.cuda.synchronize()
    prof = eng.profile_end()
    per = " ".join(f"{n.split('.')[0]}{'.' + n.split('.')[1][-1] if n.startswith('res') else ''}={ms / 3:.3f}"
                   for n, ms, c in prof)
    print(f"batch {nb}: {8 / dt:.1f} frames/s ({dt * 1e3:.3f} ms per 8 frames) | per-8-frames ms: {per}", flush=True)
