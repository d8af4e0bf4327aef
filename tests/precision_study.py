"""Per-layer precision study (CPU; test infrastructure, not collected by pytest).

Which layers of a stylization net carry the 16-bit modes' output error?  The rounding model of
oracle/bf16_layers.py is generalised to a per-layer choice of three rounding points:
  w  the layer's weights                 fp16 (RNE) or "32" (the split-fp16 pair: ~fp32)
  o  the layer's staged operand          fp16 or "32" (split hi/lo operand)
  s  the layer's stored output (y)       fp16 or "32" (fp32 storage)
and the output error of a configuration is measured against the fp32 restatement in u8 LSB
(raw output in the io_preset's 0..255 units, before truncation).

  python tests/precision_study.py --h 540 --w 960 --frames 2 [--arch johnson]

Prints, per layer and rounding point, the RMS / max raw output error when ONLY that point rounds
to fp16 (everything else fp32), the all-fp16 error, and greedy mixes (upgrade the costliest-error
points first) with their predicted error.  Used to pick the NST_DT_MIX16 layer plan.
"""
from __future__ import annotations

import argparse
import os
import sys
import time
from typing import List, Sequence, Tuple

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from oracle import bf16_layers as B  # noqa: E402
from oracle import nst_oracle as O  # noqa: E402
from neuralstyletransferv1_amd import synthetic  # noqa: E402

Spec = Sequence[Tuple[str, str, str]]  # per layer (w, o, s), each "16" or "32"


def _r(t: torch.Tensor, f: str, fmt: str) -> torch.Tensor:
    return B.rnd16(t, fmt) if f == "16" else t


def forward_mixed(arch: str, sd, x: torch.Tensor, spec: Spec, fmt: str = "fp16") -> torch.Tensor:
    """bf16_layers.forward_layers with per-layer rounding points (stats from the fp32 values)."""
    Ls = B.LAYERS[arch]
    n = x.shape[0]

    def run(i, operand):
        conv, norm, cin, cout, ks, st, axis, pad, pre = Ls[i]
        H = operand.shape[2]
        oh = {B.REFLECT_UP2: 2 * H, B.ZINSERT: 2 * H}.get(axis, (H + 2 * pre + 2 * pad - ks) // st + 1)
        return B.conv_layer(lambda idx: operand.index_select(2, idx), H, n, operand.shape[1], sd[conv + ".weight"],
                            sd[conv + ".bias"], ks, st, axis, pad, pre, spec[i][0] == "16", (0, oh), torch.float32,
                            fmt)

    def stats(i, z):
        return B.in_stats(z, sd[Ls[i][1] + ".weight"], sd[Ls[i][1] + ".bias"])

    def fill(i, y, s):  # operand of layer i from the stored y of layer i-1 (IN + ReLU)
        sc = s[..., 0][:, :, None, None].double()
        sh = s[..., 1][:, :, None, None].double()
        v = (y.double() * sc + sh).float()
        return _r(v, spec[i][1], fmt).clamp_min(0.0)

    def store(i, z):
        return _r(z, spec[i][2], fmt)

    z = run(0, _r(x, spec[0][1], fmt))
    y, s = store(0, z), stats(0, z)
    for i in (1, 2):
        z = run(i, fill(i, y, s))
        y, s = store(i, z), stats(i, z)
    nres = 4 if arch == "reconet" else 5
    relu_out = arch == "reconet"
    xv = fill(3, y, s)
    for r in range(nres):
        l1, l2 = 3 + 2 * r, 4 + 2 * r
        z1 = run(l1, xv)
        y1, s1 = store(l1, z1), stats(l1, z1)
        z2 = run(l2, fill(l2, y1, s1))
        y2, s2 = store(l2, z2), stats(l2, z2)
        v = xv + (y2 * s2[..., 0][:, :, None, None] + s2[..., 1][:, :, None, None])
        if relu_out:
            v = v.clamp_min(0.0)
        nxt = l2 + 1  # the joined stream is stored once and is the next conv's operand
        xv = _r(v, spec[nxt][1], fmt)
    u1 = 3 + 2 * nres
    z = run(u1, xv)
    y, s = store(u1, z), stats(u1, z)
    z = run(u1 + 1, fill(u1 + 1, y, s))
    y, s = store(u1 + 1, z), stats(u1 + 1, z)
    out = run(u1 + 2, fill(u1 + 2, y, s))
    if arch == "reconet":
        out = torch.tanh(out)
    if arch == "nst":
        h, w = x.shape[2:]
        ch, cw = (out.shape[2] - h) // 2, (out.shape[3] - w) // 2
        out = out[:, :, ch:ch + h, cw:cw + w]
    return out


def lsb_scale(arch: str) -> float:
    # raw output units per u8 LSB: imagenet_255 (Johnson/NST bench presets decode y/255), raw_01, tanh
    return {"johnson": 1.0, "nst": 1.0 / 255.0, "reconet": 2.0 / 255.0}[arch]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="johnson")
    ap.add_argument("--h", type=int, default=540)
    ap.add_argument("--w", type=int, default=960)
    ap.add_argument("--frames", type=int, default=2)
    ap.add_argument("--fmt", default="fp16")
    ap.add_argument("--preset", default="imagenet_255")
    ap.add_argument("--mix", default="", help="evaluate one spec: comma list of 3-char wos flags per layer "
                                              "(1 = fp16, 3 = fp32), e.g. 111,111,...")
    a = ap.parse_args()
    sd = synthetic.make_state_dict(a.arch, seed=0)
    fr = synthetic.make_frames(a.frames, a.h, a.w, seed=1000)
    x = O.encode(O.to_tensor01(fr), a.preset).float()
    nl = len(B.LAYERS[a.arch])
    names = [L[0] for L in B.LAYERS[a.arch]]
    scale = lsb_scale(a.arch)
    with torch.no_grad():
        ref = forward_mixed(a.arch, sd, x, [("32", "32", "32")] * nl).double()
        ref_u8 = B.decode_u8(ref.float(), a.preset).astype(np.int32)

        lo, hi = (0.0, 256.0) if a.arch != "reconet" else (-1.0, 1.0)

        def err(spec):
            out = forward_mixed(a.arch, sd, x, spec, a.fmt)
            d = (out.double() - ref) / scale
            # errors where both values clamp to the same end of the u8 range do not reach the frame
            live = (torch.minimum(out.double(), ref) < hi) & (torch.maximum(out.double(), ref) >= lo)
            dl = d.abs()[live]
            u8 = B.decode_u8(out, a.preset).astype(np.int32)
            du = np.abs(u8 - ref_u8)
            return (float(d.pow(2).mean().sqrt()), float(dl.max()), int(du.max()), float((du <= 1).mean()),
                    int((dl > 0.8).sum()), int((du > 1).sum()))

        if a.mix:
            flags = a.mix.split(",")
            spec = [tuple("16" if c == "1" else "32" for c in f) for f in flags]
            print(a.mix, "rms %.4f live-max %.3f u8max %d within1 %.7f n(live>0.8) %d n(u8>1) %d" % err(spec), flush=True)
            return
        t0 = time.time()
        all16 = [("16", "16", "16")] * nl
        print("all fp16: rms %.4f live-max %.3f u8max %d within1 %.7f n(live>0.8) %d n(u8>1) %d  (%.1fs)"
              % (*err(all16), time.time() - t0))
        contrib = []
        for i in range(nl):
            for k, what in enumerate("wos"):
                if what == "s" and i == nl - 1:
                    continue  # the output conv's raw value is not stored
                spec = [("32", "32", "32")] * nl
                p = list(spec[i]); p[k] = "16"; spec[i] = tuple(p)
                rms, mx = err(spec)[:2]
                contrib.append((rms * rms, i, what, mx))
                print(f"{names[i]:32s} {what}: rms {rms:.4f} max {mx:.3f}", flush=True)
        tot = sum(c[0] for c in contrib)
        print(f"sum of variances {tot:.5f} (rms {tot ** 0.5:.4f})")
        contrib.sort(reverse=True)
        acc = tot
        for v, i, what, mx in contrib:
            acc -= v
            print(f"  upgrade {names[i]:32s} {what}: var {v:.5f} ({100 * v / tot:.1f}%) -> remaining rms {max(acc, 0) ** 0.5:.4f}")


if __name__ == "__main__":
    main()
