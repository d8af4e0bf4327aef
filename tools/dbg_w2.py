"""Debug: weight-stationary stride-2 convs (conv_ws2.hip) against the generic kernel (raw output),
both measured against the fp32 path."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from dbg_wp import run

for arch, h, w in (("johnson", 64, 64), ("johnson", 70, 90), ("nst", 72, 100), ("reconet", 61, 90), ("reconet", 64, 64)):
    f = run(arch, {}, h, w, "fp32")
    g = run(arch, {"NST_NO_WS2": "1"}, h, w)
    a, b = run(arch, {}, h, w), run(arch, {}, h, w)
    s = np.abs(f).max()
    print(arch, h, w, "ws2-generic", np.abs(a - g).max() / s, "generic-fp32", np.abs(g - f).max() / s,
          "ws2-fp32", np.abs(a - f).max() / s, "det", np.abs(a - b).max(), flush=True)
