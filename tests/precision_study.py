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


def predicted_centres(arch: str, sd, in_mean: float = 0.45):
    """Per-layer, per-channel constant c the stored conv output is centred on ('P' storage): the conv's bias plus
    sum W * m over its operand's predicted channel means m -- for an operand ReLU(IN(y)) the mean of ReLU over a
    normal with IN's mean beta and std |gamma|; for the residual stream x_k the stream's mean m(x_0) + sum of
    the joined blocks' betas; for the image, in_mean (raw byte / 256 operand of the folded first layer, in
    encoded units here)."""
    from math import erf, exp, pi, sqrt
    Ls = B.LAYERS[arch]

    def relu_mean(beta, gamma):
        out = []
        for b, g in zip(beta.tolist(), gamma.tolist()):
            g = abs(g)
            if g < 1e-12:
                out.append(max(b, 0.0))
                continue
            t = b / g
            out.append(g * exp(-t * t / 2) / sqrt(2 * pi) + b * 0.5 * (1 + erf(t / sqrt(2))))
        return torch.tensor(out, dtype=torch.float64)

    def centre(i, m):
        conv = Ls[i][0]
        W, b = sd[conv + ".weight"].double(), sd[conv + ".bias"].double()
        if Ls[i][6] == B.ZINSERT:  # ConvTranspose: [cin, cout, k, k]
            return (b + (W.sum(dim=(2, 3)) * m[:, None]).sum(dim=0)).float()[None, :, None, None]
        return (b + (W.sum(dim=(2, 3)) * m[None, :]).sum(dim=1)).float()[None, :, None, None]

    def norm_mean(i):
        nm = Ls[i][1]
        return relu_mean(sd[nm + ".bias"].double(), sd[nm + ".weight"].double())

    c = [None] * len(Ls)
    c[0] = None  # the image operand's mean depends on the frame
    c[1], c[2] = centre(1, norm_mean(0)), centre(2, norm_mean(1))
    nres = 4 if arch == "reconet" else 5
    mx = norm_mean(2)
    for r in range(nres):
        l1, l2 = 3 + 2 * r, 4 + 2 * r
        c[l1] = centre(l1, mx)
        c[l2] = centre(l2, norm_mean(l1))
        mx = mx + sd[Ls[l2][1] + ".bias"].double()
    u1 = 3 + 2 * nres
    c[u1] = centre(u1, mx)
    c[u1 + 1] = centre(u1 + 1, norm_mean(u1))
    return c


def forward_mixed(arch: str, sd, x: torch.Tensor, spec: Spec, fmt: str = "fp16") -> torch.Tensor:
    """bf16_layers.forward_layers with per-layer rounding points (stats from the fp32 values)."""
    Ls = B.LAYERS[arch]
    n = x.shape[0]
    centre = predicted_centres(arch, sd)

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
        if spec[i][2] == "C":  # fp16 of the value minus its per-(frame, channel) mean (IN is shift-invariant)
            c = z.double().mean(dim=(2, 3), keepdim=True).float()
            return B.rnd16(z - c, fmt) + c
        if spec[i][2] == "P":  # ... minus a per-channel constant predicted from the weights (centre[i])
            c = centre[i]
            return B.rnd16(z - c, fmt) + c if c is not None else _r(z, "16", fmt)
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
            spec = [tuple({"1": "16", "3": "32"}.get(c, c) for c in f) for f in flags]
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
