"""Scratch: determinism of one net/dtype on a golden input — repeated forwards compared with the first and with
the oracle; on a mismatch, per-op captures of a good and a bad run give the first diverging op."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from neuralstyletransferv1_amd import synthetic  # noqa: E402
from oracle import nst_oracle as O  # noqa: E402

arch, gold, dt = sys.argv[1], sys.argv[2], sys.argv[3]
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
z = np.load(gold)
frames = z["frames"]
preset = str(z["preset"])
sd = synthetic.make_state_dict(arch, int(z["seed"]))
ref = O.stylize_u8(arch, sd, frames, preset)
m = synthetic.build_module(arch)
m.load_state_dict(sd)
m = m.cuda().eval()
m.compute_dtype = dt
fr = torch.from_numpy(frames).cuda()
outs = []
for r in range(reps):
    o = m.stylize_frames(fr, preset).cpu().numpy()
    outs.append(o)
    d = np.abs(o.astype(int) - ref.astype(int))
    print(f"rep {r}: max {d.max()} within1 {(d <= 1).mean():.6f} same_as_rep0 {np.array_equal(o, outs[0])}", flush=True)
eng = m.engine()
caps_all = []
for r in range(6):
    y, ops, caps = eng.forward_capture(fr, "u8", preset, "f32")
    caps_all.append([{k: (v.float().cpu() if v is not None else None) for k, v in c.items()} for c in caps])
for r in range(1, 6):
    for i, d in enumerate(ops):
        a, b = caps_all[0][i], caps_all[r][i]
        bad = [k for k in ("act", "res", "stats") if a.get(k) is not None and not torch.equal(a[k], b[k])]
        if bad:
            print(f"capture {r}: first diverging op {i} {d['layer']} mode {d['kernel_mode']} in {bad}", flush=True)
            break
    else:
        print(f"capture {r}: identical to capture 0", flush=True)
