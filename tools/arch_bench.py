"""Secondary timings: the three architectures (and ReCoNet(frn=True)) at 1080p, batch 8, bf16 (frames/s per GPU, HBM-resident
uint8 frames, same step as bench.py).  Not part of the bench contract; numbers quoted in DESIGN.md."""
import os, sys, time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neuralstyletransferv1_amd import synthetic

dev = torch.device("cuda", 0)
frames = torch.from_numpy(synthetic.make_frames(8, 1080, 1920, seed=5)).to(dev)
runs = [("johnson", "imagenet_255", ()), ("nst", "raw_01", ()), ("reconet", "tanh", ()), ("reconet_frn", "tanh", ()),
        ("reconet", "tanh", ("no_persistent",))]  # ReCoNet's trunk on the register-streamed kernel, for comparison
for arch, preset, ksel in runs:
    m = synthetic.build_module(arch)
    m.load_state_dict(synthetic.make_state_dict(arch, 0))
    m = m.to(dev).eval()
    m.compute_dtype = "bf16"
    m.kernel_select = frozenset(ksel)
    for _ in range(3):
        m.stylize_frames(frames, preset)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10):
        m.stylize_frames(frames, preset)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 10
    print(f"{arch}{'/' + ','.join(ksel) if ksel else ''}: {8 / dt:.1f} frames/s ({dt * 1e3:.2f} ms per batch of 8)", flush=True)
