"""Scratch: does any op read workspace bytes it did not write?  Each golden case's forward is run with the workspace
pre-filled with 0x00, 0xFF and a random pattern; outputs must be identical.  On a difference, per-op captures
under two fills name the first op whose output depends on the stale bytes."""
import glob
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from neuralstyletransferv1_amd import synthetic  # noqa: E402

dts = sys.argv[1].split(",") if len(sys.argv) > 1 else ["fp16", "bf16", "fp32", "fp32s"]
gen = torch.Generator(device="cuda").manual_seed(3)
for path in sorted(glob.glob("tests/golden/model_*.npz")):
    arch = os.path.basename(path)[len("model_"):].rsplit("_s", 1)[0]
    z = np.load(path)
    fr = torch.from_numpy(z["frames"]).cuda()
    preset = str(z["preset"])
    for dt in dts:
        m = synthetic.build_module(arch)
        m.load_state_dict(synthetic.make_state_dict(arch, int(z["seed"])))
        m = m.cuda().eval()
        m.compute_dtype = dt
        eng = m.engine()
        n, h, w, _ = fr.shape
        ws = eng.workspace(n, h, w)
        outs = {}
        for fill in ("zero", "ff", "rand"):
            if fill == "zero":
                ws.zero_()
            elif fill == "ff":
                ws.fill_(255)
            else:
                ws.copy_(torch.randint(0, 256, ws.shape, device="cuda", dtype=torch.uint8, generator=gen))
            outs[fill] = eng.stylize_u8(fr, preset).cpu()
        same = all(torch.equal(outs["zero"], o) for o in outs.values())
        msg = f"{os.path.basename(path)} {dt}: {'deterministic' if same else 'DEPENDS ON STALE WORKSPACE'}"
        if not same:
            caps = {}
            for fill in ("zero", "ff"):
                ws.zero_() if fill == "zero" else ws.fill_(255)
                y, ops, cp = eng.forward_capture(fr, "u8", preset, "f32")
                caps[fill] = [{k: (v.float().cpu() if v is not None else None) for k, v in c.items()} for c in cp]
            for i, d in enumerate(ops):
                a, b = caps["zero"][i], caps["ff"][i]
                bad = [k for k in ("act", "res", "stats") if a.get(k) is not None and not torch.equal(a[k], b[k])]
                if bad:
                    msg += f"; first op {i} {d['layer']} mode {d['kernel_mode']} {bad}"
                    break
        print(msg, flush=True)
