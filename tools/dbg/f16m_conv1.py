"""Debug: NST_DT_F16M first layer (ws9 split-weight kernel) vs the exact conv of the folded raw-byte operand."""
import sys, os
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
from neuralstyletransferv1_amd import synthetic
from oracle import bf16_layers as B

for dtype in ("fp16", "fp16m"):
    m = synthetic.build_module("johnson"); m.load_state_dict(synthetic.make_state_dict("johnson", 11))
    m = m.cuda().eval(); m.compute_dtype = dtype
    eng = m.engine()
    fr = synthetic.make_frames(2, 70, 90, seed=110)
    y, ops, caps = eng.forward_capture(torch.from_numpy(fr).cuda(), "u8", "imagenet_255", "f32")
    got = caps[0]["act"].float().cpu().permute(0, 3, 1, 2)[:, :32]
    sd = m.state_dict()
    W, b = sd["conv1.conv2d.weight"].cpu(), sd["conv1.conv2d.bias"].cpu()
    Wf, bf = B.fold_first_layer(W, b, "imagenet_255", B.REFLECT)
    x = B.raw_operand(fr, "imagenet_255").double()
    z = torch.nn.functional.conv2d(torch.nn.functional.pad(x, (4, 4, 4, 4), mode="reflect"), Wf.double()) + bf.double()[None, :, None, None]
    d = (got.double() - z).abs()
    print(dtype, ops[0]["kernel_dtype"], ops[0]["elem_bytes"], "rel", float(d.max() / z.abs().max()))
    print(" per channel max", [round(float(v), 4) for v in d.amax(dim=(0, 2, 3))])
    print(" per col (first 40)", [round(float(v), 3) for v in d.amax(dim=(0, 1, 2))[:40]])
    print(" per row (first 20)", [round(float(v), 3) for v in d.amax(dim=(0, 1, 3))[:20]])
    print(" got[0,:4,0,:4]", got[0, :4, 0, :4].tolist()); print(" ref", z[0, :4, 0, :4].tolist())
