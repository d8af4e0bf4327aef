"""Scratch: per-op comparison of the fp16 and bf16 engines on a golden input (first diverging op, NaN/inf)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from neuralstyletransferv1_amd import synthetic  # noqa: E402

arch, gold = sys.argv[1], sys.argv[2]
z = np.load(gold)
fr = torch.from_numpy(z["frames"]).cuda()
res = {}
for dt in ("bf16", "fp16"):
    m = synthetic.build_module(arch)
    m.load_state_dict(synthetic.make_state_dict(arch, int(z["seed"])))
    m = m.cuda().eval()
    m.compute_dtype = dt
    y, ops, caps = m.engine().forward_capture(fr, "u8", str(z["preset"]), "f32")
    res[dt] = (y.float().cpu(), ops, [{k: (v.float().cpu() if v is not None else None) for k, v in c.items()} for c in caps])
for i, d in enumerate(res["bf16"][1]):
    a, b = res["bf16"][2][i], res["fp16"][2][i]
    for key in ("act", "res", "stats"):
        if a.get(key) is None:
            continue
        x, y = a[key], b[key]
        for f in range(x.shape[0]):
            den = float(x[f].abs().max()) + 1e-12
            print(i, d["layer"], d["kernel_mode"], key, "frame", f, "rel", f"{float((x[f] - y[f]).abs().max()) / den:.3e}",
                  "nonfinite", int((~torch.isfinite(y[f])).sum()), "absmax", f"{float(y[f].abs().max()):.3g}")
ya, yb = res["bf16"][0], res["fp16"][0]
for f in range(ya.shape[0]):
    print("out frame", f, "rel", float((ya[f] - yb[f]).abs().max() / ya[f].abs().max()))
