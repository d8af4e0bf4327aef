"""Debug: weight-stationary trunk — determinism, fused vs unfused residual join, vs generic kernel."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neuralstyletransferv1_amd import synthetic


def net(arch, dtype="bf16"):
    m = synthetic.build_module(arch)
    m.load_state_dict(synthetic.make_state_dict(arch, 2))
    m = m.to("cuda").eval()
    m.compute_dtype = dtype
    return m


def run(env, h=70, w=90):
    for k in ("NST_NO_RESFUSE", "NST_NO_WSTAT"):
        os.environ.pop(k, None)
    for k in env:
        os.environ[k] = "1"
    m = net("johnson")
    x = torch.randn(2, 3, h, w, generator=torch.Generator().manual_seed(1)).cuda()
    return m(x).cpu().numpy(), m(x).cpu().numpy()


for h, w in ((70, 90), (64, 128)):
    fa, fb = run([], h, w)
    ua, ub = run(["NST_NO_RESFUSE"], h, w)
    ga, gb = run(["NST_NO_WSTAT"], h, w)
    g2, _ = run(["NST_NO_WSTAT", "NST_NO_RESFUSE"], h, w)
    sc = np.abs(ga).max()
    print(h, w, "det fused", np.abs(fa - fb).max(), "det unfused", np.abs(ua - ub).max(),
          "fused-unfused", np.abs(fa - ua).max() / sc, "generic fused-unfused", np.abs(ga - g2).max() / sc,
          "ws-generic", np.abs(fa - ga).max() / sc, flush=True)
