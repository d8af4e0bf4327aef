"""Debug: weight-stationary up-convs (conv_wphase.hip) against the generic phase kernel, per layer
width and fill variant (fused join / unfused), on the raw tensor output."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neuralstyletransferv1_amd import synthetic


def run(arch, env, h, w, dtype="bf16"):
    for k in ("NST_NO_RESFUSE", "NST_NO_WPHASE", "NST_WPHASE_CIN", "NST_NO_WS2"):
        os.environ.pop(k, None)
    os.environ.update(env)
    m = synthetic.build_module(arch)
    m.load_state_dict(synthetic.make_state_dict(arch, 2))
    m = m.to("cuda").eval()
    m.compute_dtype = dtype
    x = torch.randn(2, 3, h, w, generator=torch.Generator().manual_seed(1)).cuda()
    return m(x).cpu().numpy()


if __name__ == "__main__":
    for arch, h, w in (("johnson", 64, 64), ("johnson", 70, 90), ("nst", 72, 100)):
        g = run(arch, {"NST_NO_WPHASE": "1"}, h, w)
        sc = np.abs(g).max()
        for name, env in (("all", {}), ("unfused", {"NST_NO_RESFUSE": "1"}), ("cin128", {"NST_WPHASE_CIN": "128"}),
                          ("cin64", {"NST_WPHASE_CIN": "64"}), ("cin128 unfused", {"NST_WPHASE_CIN": "128", "NST_NO_RESFUSE": "1"})):
            a = run(arch, env, h, w)
            b = run(arch, env, h, w)
            print(arch, h, w, name, "rel err", np.abs(a - g).max() / sc, "det", np.abs(a - b).max(), flush=True)
