"""ORACLE — TEST INFRASTRUCTURE ONLY (imported by tests/ alone; never by the product path).

Per-layer restatement of the reference's stylization nets with the 16-bit modes' rounding points
written out (fmt "bf16": the throughput mode, NST_DT_BF16; fmt "fp16": NST_DT_F16 — the same rounding
points with IEEE binary16 round-to-nearest-even instead of bf16), for teacher-forced parity of every conv kernel: each layer is recomputed on
the CPU from the engine's OWN stored input activation (captured through nst_forward_capture), so
a layer's error is measured alone instead of accumulated over the 16 layers before it.

Layer arithmetic (the reference's, per module):
  * ConvLayer = reflection pad k//2 + Conv2d            transformer_net.py:44-54, model.py:5-15
  * InstanceNorm2d(affine, eps 1e-5, biased variance)  transformer_net.py:9 etc.
  * ResidualBlock  out = IN(conv2(relu(IN(conv1 x)))) + x  transformer_net.py:57-76
    (ReCoNet ResLayer: relu(x + branch(x)), model.py:43-60)
  * UpsampleConvLayer = nearest x2, reflect pad, conv   transformer_net.py:79-99
  * NST: ReflectionPad2d(40), zero-padded convs, ConvTranspose2d(3, s2, p1, op1), crop
                                                        transformer_net_nst.py:12-127
  * first-layer input = io_preset encode of ToTensor(frame)   pipeline.py:1445-1486

bf16 rounding points (where the engine stores or feeds bf16, include/nst_hip.h NST_DT_BF16):
  * weights: bf16(W) (RNE).  x2 up-convs run as four 2x2 sub-pixel phase convs whose weights are
    the fp64 sums of the 3x3 taps landing on one source pixel, rounded to fp32 then to bf16
    (the engine's phase packing; mathematically identical to upsample-then-conv);
  * first-layer operand: bf16(encode(x/255)) in the preset's fp32 arithmetic;
  * a conv's stored output: bf16(acc + bias), acc the fp32 sum; its IN statistics come from the
    fp32 values acc + bias (not the rounded ones);
  * the consumer's operand: bf16(fma(y, scale, shift)) then ReLU; the residual join:
    bf16(r' + (y*scale + shift)) with r' = relu(r*scale_r + shift_r) or r, fp32 ops unfused;
  * the output conv's raw fp32 value is decoded (preset) + clamped + truncated to u8.
The fp32 accumulation order differs from the engine's MFMA order, so stored bf16 values may differ
by one bf16 ulp where the fp32 sum lands near a rounding boundary, and by a few fp32 ulps of the
accumulated magnitude where the sum cancels to near zero; the tests state those bars.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F

from . import nst_oracle as O

# axis modes (same meaning as the engine's AxisMode)
REFLECT, REFLECT_UP2, ZERO, ZERO_PREREFLECT, ZINSERT = 0, 1, 2, 3, 4


def _layers_johnson():
    # transformer_net.py:4-41
    L = [("conv1.conv2d", "in1", 3, 32, 9, 1, REFLECT, 4, 0),
         ("conv2.conv2d", "in2", 32, 64, 3, 2, REFLECT, 1, 0),
         ("conv3.conv2d", "in3", 64, 128, 3, 2, REFLECT, 1, 0)]
    for r in range(1, 6):
        L += [(f"res{r}.conv1.conv2d", f"res{r}.in1", 128, 128, 3, 1, REFLECT, 1, 0),
              (f"res{r}.conv2.conv2d", f"res{r}.in2", 128, 128, 3, 1, REFLECT, 1, 0)]
    L += [("deconv1.conv2d", "in4", 128, 64, 3, 1, REFLECT_UP2, 1, 0),
          ("deconv2.conv2d", "in5", 64, 32, 3, 1, REFLECT_UP2, 1, 0),
          ("deconv3.conv2d", "", 32, 3, 9, 1, REFLECT, 4, 0)]
    return L


def _layers_nst():
    # transformer_net_nst.py:62-127
    L = [("down1.conv", "down1.norm", 3, 32, 9, 1, ZERO_PREREFLECT, 4, 40),
         ("down2.conv", "down2.norm", 32, 64, 3, 2, ZERO, 1, 0),
         ("down3.conv", "down3.norm", 64, 128, 3, 2, ZERO, 1, 0)]
    for r in range(1, 6):
        L += [(f"res{r}.conv1", f"res{r}.norm1", 128, 128, 3, 1, ZERO, 1, 0),
              (f"res{r}.conv2", f"res{r}.norm2", 128, 128, 3, 1, ZERO, 1, 0)]
    L += [("up1.conv", "up1.norm", 128, 64, 3, 1, ZINSERT, 1, 0),
          ("up2.conv", "up2.norm", 64, 32, 3, 1, ZINSERT, 1, 0),
          ("final", "", 32, 3, 9, 1, ZERO, 4, 0)]
    return L


def _layers_reconet():
    # model.py:69-116 (frn=False)
    e, d = "encoder.layers.", "decoder.layers."
    L = [(e + "0.layers.0.layers.1", e + "0.layers.1", 3, 48, 9, 1, REFLECT, 4, 0),
         (e + "1.layers.0.layers.1", e + "1.layers.1", 48, 96, 3, 2, REFLECT, 1, 0),
         (e + "2.layers.0.layers.1", e + "2.layers.1", 96, 192, 3, 2, REFLECT, 1, 0)]
    for r in range(3, 7):
        p = f"{e}{r}.branch."
        L += [(p + "0.layers.0.layers.1", p + "0.layers.1", 192, 192, 3, 1, REFLECT, 1, 0),
              (p + "1.layers.0.layers.1", p + "1.layers.1", 192, 192, 3, 1, REFLECT, 1, 0)]
    L += [(d + "1.layers.0.layers.1", d + "1.layers.1", 192, 96, 3, 1, REFLECT_UP2, 1, 0),
          (d + "3.layers.0.layers.1", d + "3.layers.1", 96, 48, 3, 1, REFLECT_UP2, 1, 0),
          (d + "4.layers.0.layers.1", "", 48, 3, 9, 1, REFLECT, 4, 0)]
    return L


LAYERS = {"johnson": _layers_johnson(), "nst": _layers_nst(), "reconet": _layers_reconet()}


def bf16(t: torch.Tensor) -> torch.Tensor:
    """Round fp32 values to bf16 (round to nearest even) and back."""
    return t.to(torch.bfloat16).to(torch.float32)


TORCH16 = {"bf16": torch.bfloat16, "fp16": torch.float16}


def rnd16(t: torch.Tensor, fmt: str = "bf16") -> torch.Tensor:
    """Round fp32 values to the 16-bit format fmt (round to nearest even) and back."""
    return t.to(TORCH16[fmt]).to(torch.float32)


def bf16_ulp_diff(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """|a - b| in ulps of their 16-bit format (both bf16 or both fp16 tensors; sign-magnitude
    patterns mapped to ordered integers; +0 == -0)."""
    def ordered(t):
        i = t.contiguous().view(torch.int16).to(torch.int32)
        return torch.where(i < 0, -(i & 0x7FFF), i)
    return (ordered(a) - ordered(b)).abs()


# ------------------------------------------------------------------------- the consumer's fill
def fill_operand(y: torch.Tensor, ys: Optional[torch.Tensor], in_relu: bool, r: Optional[torch.Tensor] = None,
                 rs: Optional[torch.Tensor] = None, relu_out: bool = False, round_bf16: bool = True,
                 fmt: str = "bf16") -> torch.Tensor:
    """The conv input the engine stages: y [n,c,h,w] (stored values), ys [n,c,2] {scale, shift}.
    No residual: fma(y, scale, shift) rounded once to fp32 (then bf16), ReLU.  Residual join
    (ResidualBlock): r' + (y*scale + shift) in unfused fp32, r' = relu(r*scale_r + shift_r) if rs
    (bf16: r' = the normalised fill of r, rounded to bf16 — block 1's input x_0 as the trunk stores
    it, conv_wstat.hip XO)."""
    rnd = (lambda t: rnd16(t, fmt)) if round_bf16 else (lambda t: t)
    if r is None:
        if ys is None:
            return y
        sc = ys[..., 0][:, :, None, None].double()
        sh = ys[..., 1][:, :, None, None].double()
        v = (y.double() * sc + sh).float()  # fma: exact product (bf16 x fp32), one rounding
        v = rnd(v)
        return v.clamp_min(0.0) if in_relu else v
    sc, sh = ys[..., 0][:, :, None, None], ys[..., 1][:, :, None, None]
    rr = r
    if rs is not None:
        if round_bf16:  # r' exactly as a normalising fill stages it (the stored x_0 of the fused trunk)
            rr = fill_operand(r, rs, True, round_bf16=True, fmt=fmt)
        else:
            rr = (r * rs[..., 0][:, :, None, None] + rs[..., 1][:, :, None, None]).clamp_min(0.0)
    v = rr + (y * sc + sh)
    if relu_out:
        v = v.clamp_min(0.0)
    return rnd(v)


# io_preset encode constants as the engine rounds them to fp32 (nst_api.cpp preset_consts; pipeline.py:1445-1486):
# x_c = ((byte[perm c] / 255) * a_c - b_c) / d_c
def _f32(v):
    return float(np.float32(v))


PRESET_ENC = {
    "tanh": ((2.0,) * 3, (1.0,) * 3, (1.0,) * 3, (0, 1, 2)),
    "imagenet_01": ((1.0,) * 3, tuple(_f32(m) for m in (0.485, 0.456, 0.406)), tuple(_f32(s) for s in (0.229, 0.224, 0.225)),
                    (0, 1, 2)),
    "imagenet_255": ((255.0,) * 3, tuple(_f32(np.float32(m) * np.float32(255.0)) for m in (0.485, 0.456, 0.406)),
                     tuple(_f32(np.float32(s) * np.float32(255.0)) for s in (0.229, 0.224, 0.225)), (0, 1, 2)),
    "caffe_bgr": ((255.0,) * 3, tuple(_f32(c) for c in (103.939, 116.779, 123.68)), (1.0,) * 3, (2, 1, 0)),
    "raw_255": ((255.0,) * 3, (0.0,) * 3, (1.0,) * 3, (0, 1, 2)),
    "raw_01": ((1.0,) * 3, (0.0,) * 3, (1.0,) * 3, (0, 1, 2)),
}


def fold_first_layer(W: torch.Tensor, b: torch.Tensor, preset: str, axis: int):
    """The engine's first layer over uint8 frames (nst_api.cpp fold_first_layer): operand o_c = byte[perm c] / 256
    (exact), W'[.][c] = W * 256 a_c / (255 d_c), bias' = bias - sum W b_c / d_c (fp64 -> fp32), or None where the
    fold does not hold (zero padding with b != 0)."""
    if preset not in PRESET_ENC:
        return None
    a, bb, d, _ = PRESET_ENC[preset]
    if axis != REFLECT and any(v != 0.0 for v in bb):
        return None
    Wd = W.double()
    sc = torch.tensor([256.0 * a[c] / (255.0 * d[c]) for c in range(3)], dtype=torch.float64)
    sh = torch.tensor([bb[c] / d[c] for c in range(3)], dtype=torch.float64)
    Wf = (Wd * sc[None, :, None, None]).float()
    bf = (b.double() - (Wd * sh[None, :, None, None]).sum(dim=(1, 2, 3))).float()
    return Wf, bf


def raw_operand(frames_u8: np.ndarray, preset: str) -> torch.Tensor:
    """The staged first-layer operand with the fold: [n,3,h,w] byte[perm c] / 256 (exact in bf16 / fp16)."""
    perm = list(PRESET_ENC[preset][3])
    x = torch.from_numpy(np.ascontiguousarray(frames_u8)).permute(0, 3, 1, 2).float()
    return x[:, perm] / 256.0


def encode_operand(frames_u8: np.ndarray, preset: str, round_bf16: bool = True, fmt: str = "bf16") -> torch.Tensor:
    """First-layer operand: encode(ToTensor(frame)) in the preset's fp32 arithmetic (+ 16-bit rounding)."""
    v = O.encode(O.to_tensor01(frames_u8), preset).float()
    return rnd16(v, fmt) if round_bf16 else v


# ------------------------------------------------------------------------- conv emulation
def _pad(x: torch.Tensor, axis: int, pad: int, pre: int) -> torch.Tensor:
    if axis == REFLECT:
        return F.pad(x, (pad,) * 4, mode="reflect")
    if axis == ZERO:
        return F.pad(x, (pad,) * 4)
    if axis == ZERO_PREREFLECT:
        return F.pad(F.pad(x, (pre,) * 4, mode="reflect"), (pad,) * 4)
    raise ValueError(axis)


def phase_weights(W: torch.Tensor, convT: bool, round_bf16: bool, fmt: str = "bf16") -> torch.Tensor:
    """[2,2,cout,cin,2,2] sub-pixel phase weights of a x2 up-conv (fp64 sums of the taps landing on
    one source pixel, then fp32 (and bf16)): output (2y+a, 2x+b) = sum_t Wp[a,b,:,:,ty,tx] *
    S[y + off_a + ty, x + off_b + tx], off = a - 1 for nearest x2 (clamped source), 0 for
    ConvTranspose2d(s2, p1, op1) (zeros past the edge)."""
    Wd = W.double()

    def taps(a, t):
        if convT:
            if a == 0:
                return [1] if t == 0 else []
            return [2] if t == 0 else [0]
        if a == 0:
            return [0] if t == 0 else [1, 2]
        return [0, 1] if t == 0 else [2]
    if convT:
        cin, cout = W.shape[0], W.shape[1]
    else:
        cout, cin = W.shape[0], W.shape[1]
    out = torch.zeros(2, 2, cout, cin, 2, 2, dtype=torch.float64)
    for a in range(2):
        for b in range(2):
            for ty in range(2):
                for tx in range(2):
                    for ky in taps(a, ty):
                        for kx in taps(b, tx):
                            if convT:
                                out[a, b, :, :, ty, tx] += Wd[:, :, ky, kx].t()
                            else:
                                out[a, b, :, :, ty, tx] += Wd[:, :, ky, kx]
    out = out.float()
    return rnd16(out, fmt) if round_bf16 else out


def _reflect_idx(v: np.ndarray, L: int) -> np.ndarray:
    v = np.abs(v)
    return np.where(v >= L, 2 * L - 2 - v, v)


def source_rows(axis: int, u: np.ndarray, L: int, pad: int, pre: int) -> np.ndarray:
    """Source index (or -1 = zero) of padded-grid index u along one axis of a plain conv."""
    v = u - pad
    if axis == REFLECT:
        return _reflect_idx(v, L)
    if axis == ZERO:
        return np.where((v < 0) | (v >= L), -1, v)
    if axis == ZERO_PREREFLECT:
        inside = (v >= 0) & (v < L + 2 * pre)
        return np.where(inside, _reflect_idx(np.clip(v - pre, -L + 1, 2 * L - 2), L), -1)
    raise ValueError(axis)


def _gather(get_rows, idx: np.ndarray, n: int, c: int) -> torch.Tensor:
    """Operand rows idx (-1 -> zero rows): get_rows(valid source rows) -> [n,c,k,w]."""
    valid = idx >= 0
    rows = get_rows(torch.from_numpy(np.where(valid, idx, 0)).long())
    if not valid.all():
        rows = rows * torch.from_numpy(valid.astype(np.float32))[None, None, :, None]
    return rows


def _pad_cols(x: torch.Tensor, axis: int, pad: int, pre: int) -> torch.Tensor:
    if axis == REFLECT:
        return F.pad(x, (pad, pad, 0, 0), mode="reflect")
    if axis == ZERO:
        return F.pad(x, (pad, pad, 0, 0))
    if axis == ZERO_PREREFLECT:
        return F.pad(F.pad(x, (pre, pre, 0, 0), mode="reflect"), (pad, pad, 0, 0))
    raise ValueError(axis)


def conv_layer(get_rows, H: int, n: int, c: int, W: torch.Tensor, b: torch.Tensor, ks: int, stride: int, axis: int,
               pad: int, pre: int, round_bf16: bool, rows: Tuple[int, int], acc: torch.dtype = torch.float32,
               fmt: str = "bf16") -> torch.Tensor:
    """Output rows rows[0]..rows[1]-1 of one conv of the net -> fp32 acc + bias [n,cout,k,ow] (before
    rounding).  get_rows(src_row_indices) returns the staged operand rows [n,c,k,w] (fill applied);
    H = source height.  Up-convs need even row bounds."""
    r0, r1 = rows
    if axis in (REFLECT_UP2, ZINSERT):
        convT = axis == ZINSERT
        Wp = phase_weights(W, convT, round_bf16, fmt).to(acc)
        y0, y1 = r0 // 2, r1 // 2
        u = np.arange(y0 - 1, y1 + 1)  # source rows y0-1 .. y1 (one row of halo each side)
        idx = np.where((u < 0) | (u >= H), -1, u) if convT else np.clip(u, 0, H - 1)
        S = _gather(get_rows, idx, n, c)
        S = (F.pad(S, (1, 1, 0, 0)) if convT else F.pad(S, (1, 1, 0, 0), mode="replicate")).to(acc)
        w = S.shape[-1] - 2
        out = torch.empty(n, Wp.shape[2], 2 * (y1 - y0), 2 * w, dtype=acc)
        for a in range(2):
            for bb in range(2):
                oa = 0 if convT else a - 1
                ob = 0 if convT else bb - 1
                src = S[:, :, oa + 1:oa + 1 + (y1 - y0) + 1, ob + 1:ob + 1 + w + 1]
                out[:, :, a::2, bb::2] = F.conv2d(src, Wp[a, bb])
        return out.float() + b.float()[None, :, None, None]
    Wr = (rnd16(W, fmt) if round_bf16 else W).to(acc)
    u = np.arange(r0 * stride, (r1 - 1) * stride + ks)
    P = _gather(get_rows, source_rows(axis, u, H, pad, pre), n, c)
    P = _pad_cols(P, axis, pad, pre).to(acc)
    y = F.conv2d(P, Wr, stride=stride)
    return y.float() + b.float()[None, :, None, None]


def forward_layers(arch: str, sd: Dict[str, torch.Tensor], x: torch.Tensor, round_bf16: bool = False,
                   acc: torch.dtype = torch.float32, fmt: str = "bf16") -> torch.Tensor:
    """The whole net through this module's per-layer functions (x = encoded input [n,3,h,w]):
    with round_bf16=False it restates the reference forward (checked against nst_oracle.forward);
    with True it is the bf16 mode's rounding model end to end (stats from the fp32 values)."""
    Ls = LAYERS[arch]
    n = x.shape[0]

    def run(i, operand):
        conv, norm, cin, cout, ks, st, axis, pad, pre = Ls[i]
        H = operand.shape[2]
        oh = {REFLECT_UP2: 2 * H, ZINSERT: 2 * H}.get(axis, (H + 2 * pre + 2 * pad - ks) // st + 1)
        return conv_layer(lambda idx: operand.index_select(2, idx), H, n, operand.shape[1], sd[conv + ".weight"],
                          sd[conv + ".bias"], ks, st, axis, pad, pre, round_bf16, (0, oh), acc, fmt)

    rnd = (lambda t: rnd16(t, fmt)) if round_bf16 else (lambda t: t)

    def stats(i, z):
        return in_stats(z, sd[Ls[i][1] + ".weight"], sd[Ls[i][1] + ".bias"])

    op = rnd(x) if round_bf16 else x
    z = run(0, op)
    y, s = rnd(z), stats(0, z)
    for i in (1, 2):
        z = run(i, fill_operand(y, s, True, round_bf16=round_bf16, fmt=fmt))
        y, s = rnd(z), stats(i, z)
    nres = 4 if arch == "reconet" else 5
    relu_out = arch == "reconet"
    xs, xst = y, s  # the residual stream: block 1's input is relu(IN(conv3)), applied lazily
    xv = fill_operand(xs, xst, True, round_bf16=round_bf16, fmt=fmt)
    for r in range(nres):
        l1, l2 = 3 + 2 * r, 4 + 2 * r
        z1 = run(l1, xv)
        y1, s1 = rnd(z1), stats(l1, z1)
        z2 = run(l2, fill_operand(y1, s1, True, round_bf16=round_bf16, fmt=fmt))
        y2, s2 = rnd(z2), stats(l2, z2)
        xv = fill_operand(y2, s2, False, r=xv, relu_out=relu_out, round_bf16=round_bf16, fmt=fmt)
    u1 = 3 + 2 * nres
    z = run(u1, xv)
    y, s = rnd(z), stats(u1, z)
    z = run(u1 + 1, fill_operand(y, s, True, round_bf16=round_bf16, fmt=fmt))
    y, s = rnd(z), stats(u1 + 1, z)
    out = run(u1 + 2, fill_operand(y, s, True, round_bf16=round_bf16, fmt=fmt))
    if arch == "reconet":
        out = torch.tanh(out)
    if arch == "nst":
        h, w = x.shape[2:]
        ch, cw = (out.shape[2] - h) // 2, (out.shape[3] - w) // 2
        out = out[:, :, ch:ch + h, cw:cw + w]
    return out


def in_stats(z: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float = 1e-5) -> torch.Tensor:
    """{scale, shift} [n,c,2] of InstanceNorm2d(affine) over z's spatial extent (biased variance)."""
    zd = z.double()
    mean = zd.mean(dim=(2, 3))
    var = (zd * zd).mean(dim=(2, 3)) - mean * mean
    scale = gamma.double()[None, :] / torch.sqrt(var.clamp_min(0.0) + eps)
    shift = beta.double()[None, :] - mean * scale
    return torch.stack([scale, shift], dim=-1).float()


def decode_u8(y: torch.Tensor, preset: str) -> np.ndarray:
    """Raw output -> io_preset decode + clamp(0,1) -> ToPILImage truncation (NHWC u8)."""
    return O.to_pil_u8(O.decode(y, preset))
