"""Teacher-forced per-layer parity of the 16-bit engine modes, bf16 and fp16 (helper of
tests/test_gpu_layers.py).

Runs one batch through nst_forward_capture, then recomputes every op on the CPU from the engine's
own stored inputs (oracle/bf16_layers.py) and compares:
  * each conv's stored 16-bit output element-wise, in ulps of its format;
  * each conv's InstanceNorm {scale, shift} (from the engine's fp32 values) against the statistics
    of the oracle's fp32 values;
  * each joined residual stream bit for bit;
  * the output conv's raw fp32 values and its decoded u8 frames.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from oracle import bf16_layers as B

# bars (tests state them; see oracle/bf16_layers.py for why they are not zero)
ULP_MAX = 1              # stored bf16 outputs: at most one bf16 ulp apart ...
ATOL_REL = 4e-6          # ... or within this fraction of the layer's max |value| (sums that cancel to ~0)
ULP1_FRAC_MAX = 1e-3     # at most 0.1 % of the elements one ulp apart (accumulation-order rounding flips)
# fp16's ulp is 8x finer than bf16's, so the same fp32 accumulation-order differences flip its
# rounding ~8x as often: at most 0.8 % of the elements one fp16 ulp apart
ULP1_FRAC_MAX_F16 = 8e-3
STATS_REL = 1e-5         # IN scale/shift vs the oracle's statistics of its fp32 values (measured <= 4e-7)
RAW_REL = 5e-6           # output conv raw fp32, relative to max |y| (measured <= 1.1e-6)
U8_EXACT_MIN = 0.9999    # decoded u8 frames: >= 99.99 % identical, the rest 1 LSB (truncation boundary)
# split-precision layers (NST_DT_F16M: fp16 hi / lo operand and weight pairs, ~22-bit products, fp32 output) against
# the exact (fp64) conv of the same fp32 operand: within this fraction of the layer's max |value|
SPLIT_REL = 2e-5
SPLIT_KDT = (3, 16, 17, 18, 19, 20)  # NST_DT_F32S and the NST_KDT_* split kernels (nst_op_desc.kernel_dtype)
KDT_SPLITO = 20  # split operand, fp16 weights (conv_ws1s.hip): the weights keep their fp16 rounding


def _nchw(t: torch.Tensor, c: int) -> torch.Tensor:
    return t[..., :c].float().cpu().permute(0, 3, 1, 2).contiguous()


def _frn_tau_names(li: int):
    """ReCoNet(frn=True) (model.py with frn.py): the TLU threshold each layer's conv reads (its bias
    absorbs sum W tau) and the ones its FRN shift absorbs, as nst_api.cpp frn_layer folds them."""
    def act_tau(l):
        if l <= 2:
            return f"encoder.layers.{l}.layers.2.tau"
        if l <= 10:
            return f"encoder.layers.{3 + (l - 3) // 2}.branch.0.layers.2.tau"
        return "decoder.layers.1.layers.2.tau" if l == 11 else "decoder.layers.3.layers.2.tau"

    def block_tau(r):
        return f"encoder.layers.{3 + r}.activation.tau"

    def stream_tau(r):
        return act_tau(2) if r == 0 else block_tau(r - 1)
    in_tau = None
    if li in (1, 2):
        in_tau = act_tau(li - 1)
    elif 3 <= li <= 10:
        in_tau = stream_tau((li - 3) // 2) if (li - 3) % 2 == 0 else act_tau(li - 1)
    elif li == 11:
        in_tau = block_tau(3)
    elif li >= 12:
        in_tau = act_tau(li - 1)
    join = 3 <= li <= 10 and (li - 3) % 2 == 1
    own = block_tau((li - 3) // 2) if join else (act_tau(li) if li <= 12 else None)
    prev = stream_tau((li - 3) // 2) if join else None
    return in_tau, own, prev


def _frn_bias(sd, li, W, b):
    in_tau = _frn_tau_names(li)[0]
    if in_tau is None:
        return b
    t = sd[in_tau].double().flatten()
    return (b.double() + (W.double().sum(dim=(2, 3)) * t[None, :]).sum(dim=1)).float()


def _frn_stats(sd, li, norm, z):
    """{gamma * rsqrt(mean(z^2) + |eps|), beta - tau_own (+ tau_prev on a join)} (frn.py:71-78)."""
    _, own, prev = _frn_tau_names(li)
    zd = z.double()
    nu2 = (zd * zd).mean(dim=(2, 3))
    eps = abs(float(sd[norm + ".eps"][0]))
    scale = sd[norm + ".weight"].double().flatten()[None, :] / torch.sqrt(nu2 + eps)
    shift = sd[norm + ".bias"].double().flatten() - sd[own].double().flatten()
    if prev is not None:
        shift = shift + sd[prev].double().flatten()
    return torch.stack([scale, shift[None, :].expand_as(scale)], dim=-1).float()


def check_layers(net, frames_u8: np.ndarray, preset: str, bands: Optional[Sequence[Tuple[float, int]]] = None,
                 acc: torch.dtype = torch.float32) -> List[Dict]:
    """-> one record per op.  bands: None = every output row; else [(fraction, rows)] row bands
    (start = fraction of the output height, rounded down to even) checked per op (4K frames)."""
    arch = {0: "johnson", 1: "nst", 2: "reconet", 3: "reconet_frn"}[net.ARCH]
    fmt = "fp16" if net.compute_dtype in ("fp16", "float16", "fp16m") else "bf16"
    ulp1_max = ULP1_FRAC_MAX_F16 if fmt == "fp16" else ULP1_FRAC_MAX
    frn = arch == "reconet_frn"
    sd = {k: v.detach().float().cpu() for k, v in net.state_dict().items()}
    eng = net.engine()
    fr_dev = torch.from_numpy(frames_u8).to(eng.device)
    n, H0, W0, _ = frames_u8.shape
    oh, ow = eng.output_hw(H0, W0)
    y_raw, ops, caps = eng.forward_capture(fr_dev, "u8", preset, "f32")
    y_raw = y_raw.cpu()
    y_u8 = None
    if (oh, ow) == (H0, W0):
        y_u8, _, _ = eng.forward_capture(fr_dev, "u8", preset, "u8")
        y_u8 = y_u8.cpu().numpy()
    torch.cuda.synchronize()
    layers = B.LAYERS["reconet" if frn else arch]
    host = [{k: (v.cpu() if v is not None else None) for k, v in c.items()} for c in caps]
    writer: Dict[int, Tuple[int, str]] = {}   # buffer -> (op, "act" | "res")
    layer_op: Dict[int, int] = {}            # layer -> conv op that ran it (its stats capture)
    recs = []
    x_enc = None
    for i, d in enumerate(ops):
        conv, norm, cin, cout, ks, st, axis, pad, pre = layers[d["layer"]]
        split = d["kernel_dtype"] in SPLIT_KDT
        if d["kind"] != 0:
            # NST_DT_F16M's first residual join (fp32 y and r -> the fp16 stream): the fp32 arithmetic of the
            # reference's ResidualBlock (product, then sum), one fp16 rounding
            if d["in_elem_bytes"] != 4:
                raise AssertionError("only the split-precision program has a separate residual op")
            j, kind = writer[d["src"]]
            y = _nchw(host[j][kind], cout)
            jr, kr = writer[d["res_buf"]]
            r = _nchw(host[jr][kr], cout)
            ys = host[layer_op[d["in_norm"]]]["stats"][:, :cout]
            if d["res_norm"] >= 0:
                rs = host[layer_op[d["res_norm"]]]["stats"][:, :cout]
                r = r * rs[..., 0][:, :, None, None] + rs[..., 1][:, :, None, None]
                r = r.clamp_min(0.0)
            v = r + (y * ys[..., 0][:, :, None, None] + ys[..., 1][:, :, None, None])
            if d["relu_out"]:
                v = v.clamp_min(0.0)
            got = host[i]["act"].permute(0, 3, 1, 2)[:, :cout].contiguous()
            rec = {"op": i, "layer": conv + " (join)", "mode": -1, "elements": v.numel()}
            if d["elem_bytes"] == 2:  # the fp16 stream
                ulp = B.bf16_ulp_diff(got, v.to(torch.float16))
                rec.update(ulp_max=int(ulp.max()), ulp1_frac=float((ulp >= 1).float().mean()))
                assert rec["ulp_max"] <= 1 and rec["ulp1_frac"] <= 1e-4, rec
            else:  # fp32 stream: the same fp32 operations
                rec["rel"] = float((got - v).abs().max() / v.abs().max().clamp_min(1e-12))
                assert rec["rel"] <= 1e-6, rec
            writer[d["dst"]] = (i, "act")
            recs.append(rec)
            continue

        def stats_of(layer):
            return host[layer_op[layer]]["stats"][:, :, :]

        def buf_rows(buf):
            j, kind = writer[buf]
            return _nchw(host[j][kind], cin)

        W, bias = sd[conv + ".weight"], sd[conv + ".bias"]
        folded = B.fold_first_layer(W, bias, preset, axis) if d["src"] == -1 else None
        if d["src"] == -1:
            if folded is not None:  # uint8 frames: raw bytes / 256 and the encode in the weights (nst_api.cpp)
                W, bias = folded
                src = B.raw_operand(frames_u8, preset)
            else:
                if x_enc is None:
                    x_enc = B.encode_operand(frames_u8, preset, fmt=fmt)
                src = x_enc
            if split:
                src = src.double()

            def get_rows(idx, src=src):
                return src.index_select(2, idx)
            Hs = src.shape[2]
        else:
            ysrc = buf_rows(d["src"])
            ys = stats_of(d["in_norm"])[:, :cin] if d["in_norm"] >= 0 else None
            r = rs = None
            if d["res_buf"] >= 0:
                r = buf_rows(d["res_buf"])
                rs = stats_of(d["res_norm"])[:, :cin] if d["res_norm"] >= 0 else None

            def get_rows(idx, ysrc=ysrc, ys=ys, r=r, rs=rs, d=d, split=split):
                v = B.fill_operand(ysrc.index_select(2, idx), ys, bool(d["in_relu"]),
                                   None if r is None else r.index_select(2, idx), rs, bool(d["relu_out"]),
                                   round_bf16=not split, fmt=fmt)
                return v.double() if split else v
            Hs = ysrc.shape[2]
            if d["res_out"] >= 0:  # the joined stream the op wrote for its own pixels: bit-exact
                joined = get_rows(torch.arange(Hs))
                got = _nchw(host[i]["res"], cin)
                if not torch.equal(got, joined):
                    bad = (got != joined).nonzero()
                    ex = []
                    for q in bad[:6].tolist():
                        b_, c_, y_, x_ = q
                        ex.append({"at": q, "got": float(got[b_, c_, y_, x_]), "want": float(joined[b_, c_, y_, x_]),
                                   "y": float(ysrc[b_, c_, y_, x_]),
                                   "r": None if r is None else float(r[b_, c_, y_, x_]),
                                   "ys": ys[b_, c_].tolist(), "rs": None if rs is None else rs[b_, c_].tolist()})
                    raise AssertionError(f"op {i} ({conv}): joined residual stream differs at {bad.shape[0]} of "
                                         f"{got.numel()} values (nan got {int(got.isnan().sum())} want "
                                         f"{int(joined.isnan().sum())}); {ex}")
        final = d["dst"] == -2
        ch = d["conv_h"]
        row_sets = [(0, ch)] if bands is None else sorted({
            (r0, min(ch, r0 + k)) for f, k in bands for r0 in [min(max(0, int(f * ch)) // 2 * 2, max(0, ch - k) // 2 * 2)]})
        rec = {"op": i, "layer": conv, "mode": d["kernel_mode"], "elements": 0}
        if frn:  # TLU outputs are stored shifted by -tau: the bias absorbs sum W tau
            bias = _frn_bias(sd, d["layer"], W, bias)
        for (r0, r1) in row_sets:
            wround = not split or d["kernel_dtype"] == KDT_SPLITO
            z = B.conv_layer(get_rows, Hs, n, cin, W, bias, ks, st, axis, pad, pre, wround, (r0, r1),
                             torch.float64 if split else acc, fmt)
            if final:
                if arch.startswith("reconet"):
                    z = torch.tanh(z)
                cy, cx = (d["conv_h"] - d["out_h"]) // 2, (d["conv_w"] - d["out_w"]) // 2
                lo, hi = max(r0, cy), min(r1, cy + d["out_h"])
                if hi <= lo:
                    continue
                zc = z[:, :, lo - r0:hi - r0, cx:cx + d["out_w"]]
                yc = y_raw[:, :, lo - cy:hi - cy, :]
                rel = float((yc - zc).abs().max() / zc.abs().max().clamp_min(1e-12))
                rec["raw_rel"] = max(rec.get("raw_rel", 0.0), rel)
                assert rel <= RAW_REL, f"op {i} ({conv}) raw output rel err {rel:.2e} rows {r0}:{r1}"
                if y_u8 is not None:
                    ref = B.decode_u8(zc, preset)
                    got = y_u8[:, lo - cy:hi - cy]
                    dd = np.abs(got.astype(int) - ref.astype(int))
                    rec["u8_max"] = max(rec.get("u8_max", 0), int(dd.max()))
                    rec["u8_exact"] = min(rec.get("u8_exact", 1.0), float((dd == 0).mean()))
                    assert dd.max() <= 1 and (dd == 0).mean() >= U8_EXACT_MIN, (i, conv, dd.max(), (dd == 0).mean())
                rec["elements"] += zc.numel()
                continue
            got_full = host[i]["act"]
            rec["absmax"] = max(rec.get("absmax", 0.0), float(got_full.float().abs().max()))
            got = got_full[:, r0:r1].permute(0, 3, 1, 2)[:, :cout].contiguous()
            pad_ch = got_full[:, r0:r1, :, cout:]
            assert (pad_ch.float() == 0).all(), f"op {i} ({conv}): padded channels not zero"
            if split:  # fp32 (or fp16) output of ~22-bit products vs the exact conv
                zr = z if d["elem_bytes"] == 4 else z.to(torch.float16).float()
                rel = float((got.float() - zr.float()).abs().max() / zr.abs().max().clamp_min(1e-12))
                rec["elements"] += zr.numel()
                rec["split_rel"] = max(rec.get("split_rel", 0.0), rel)
                lim = SPLIT_REL if d["elem_bytes"] == 4 else 1e-3
                assert rel <= lim, f"op {i} ({conv}) rows {r0}:{r1}: split-precision output rel err {rel:.2e} > {lim}"
                if bands is None:
                    s_ref = B.in_stats(z.float(), sd[norm + ".weight"], sd[norm + ".bias"])
                    s_got = host[i]["stats"][:, :cout]
                    err = (s_got - s_ref).abs() / s_ref.abs().amax(dim=1, keepdim=True).clamp_min(1e-6)
                    rec["stats_rel"] = float(err.max())
                    assert rec["stats_rel"] <= STATS_REL, (i, conv, rec["stats_rel"])
                continue
            ref = z.to(B.TORCH16[fmt])
            ulp = B.bf16_ulp_diff(got, ref)
            diff = (got.float() - ref.float()).abs()
            atol = ATOL_REL * float(ref.float().abs().max())
            bad = (ulp > ULP_MAX) & (diff > atol)
            rec["elements"] += ref.numel()
            rec["ulp1_frac"] = max(rec.get("ulp1_frac", 0.0), float((ulp >= 1).float().mean()))
            rec["ulp_max"] = max(rec.get("ulp_max", 0), int(ulp.max()))
            rec["bad"] = rec.get("bad", 0) + int(bad.sum())
            assert not bad.any(), (f"op {i} ({conv}) rows {r0}:{r1}: {int(bad.sum())} elements beyond "
                                   f"{ULP_MAX} ulp / atol {atol:.2e}; first at {tuple(bad.nonzero()[0].tolist())}")
            assert rec["ulp1_frac"] <= ulp1_max, (i, conv, rec["ulp1_frac"])
            if bands is None:  # statistics need the whole frame
                s_ref = (_frn_stats(sd, d["layer"], norm, z) if frn else
                         B.in_stats(z, sd[norm + ".weight"], sd[norm + ".bias"]))
                s_got = host[i]["stats"][:, :cout]
                err = (s_got - s_ref).abs() / s_ref.abs().amax(dim=1, keepdim=True).clamp_min(1e-6)
                rec["stats_rel"] = float(err.max())
                assert rec["stats_rel"] <= STATS_REL, (i, conv, rec["stats_rel"])
        if not final:
            writer[d["dst"]] = (i, "act")
            layer_op[d["layer"]] = i
            if d["res_out"] >= 0:
                writer[d["res_out"]] = (i, "res")
        recs.append(rec)
    return recs
