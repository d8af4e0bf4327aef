"""Stream-split experiment: the configs[1] batch of 8 1080p frames as ONE nst_forward of 8 frames, against the same
8 frames as S sub-batches (8 / S frames each) issued on S HIP streams with separate workspaces, so one sub-batch's
launch gaps and kernel tails can be filled by another's kernels.  Outputs must be identical (frames are independent).
  python tools/stream_split_bench.py [arch] [dtype]    -> one JSON line"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neuralstyletransferv1_amd import _lib, synthetic  # noqa: E402
from neuralstyletransferv1_amd._lib import check, lib  # noqa: E402

arch = sys.argv[1] if len(sys.argv) > 1 else "johnson"
dt = sys.argv[2] if len(sys.argv) > 2 else "bf16"
dev = torch.device("cuda", 0)
N, H, W = 8, 1080, 1920
frames = torch.from_numpy(synthetic.make_frames(N, H, W, seed=5)).to(dev)
m = synthetic.build_module(arch)
m.load_state_dict(synthetic.make_state_dict(arch, 0))
m = m.to(dev).eval()
m.compute_dtype = dt
eng = m.engine(dev)
eng.set_stream_split(1)  # the manual split below; the library's own split (nst_set_stream_split) is timed after it
pid = _lib.PRESETS["imagenet_255"]


def ws_bytes(n):
    need = _lib.ctypes.c_size_t()
    check(lib().nst_workspace_bytes(eng._h, n, H, W, _lib.ctypes.byref(need)), "nst_workspace_bytes")
    return need.value


out = {"arch": arch, "dtype": dt}
ref = None
for S in (1, 2, 4):
    n = N // S
    streams = [torch.cuda.Stream(dev) for _ in range(S)]
    wss = [torch.empty(ws_bytes(n), dtype=torch.uint8, device=dev) for _ in range(S)]
    y = torch.empty((N, H, W, 3), dtype=torch.uint8, device=dev)

    def step():
        main = torch.cuda.current_stream(dev)
        ev = torch.cuda.Event()
        ev.record(main)
        for i, s in enumerate(streams):
            s.wait_event(ev)
            check(lib().nst_forward(eng._h, frames[i * n].data_ptr(), _lib.NST_IO_U8_NHWC, n, H, W, pid,
                                    y[i * n].data_ptr(), _lib.NST_IO_U8_NHWC, wss[i].data_ptr(), wss[i].numel(),
                                    s.cuda_stream), "nst_forward")
        for s in streams:
            main.wait_stream(s)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    K = 20
    t0 = time.perf_counter()
    for _ in range(K):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / K * 1e3
    if ref is None:
        ref = y.clone()
    out[f"split_{S}"] = {"ms_per_step": round(ms, 3), "frames_per_s": round(N / ms * 1e3, 1),
                         "identical": bool(torch.equal(y, ref))}
for k in (1, 2, 3, 4):
    eng.set_stream_split(k)
    for _ in range(3):
        y2 = eng.stylize_u8(frames, "imagenet_255")
    torch.cuda.synchronize()
    K = 20
    t0 = time.perf_counter()
    for _ in range(K):
        y2 = eng.stylize_u8(frames, "imagenet_255")
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / K * 1e3
    out[f"lib_split_{k}"] = {"ms_per_step": round(ms, 3), "frames_per_s": round(N / ms * 1e3, 1),
                             "identical": bool(torch.equal(y2, ref))}
print(json.dumps(out))
