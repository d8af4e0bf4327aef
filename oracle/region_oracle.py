"""CPU oracle of the region-blend compositor (region_blend.py) -- TEST INFRASTRUCTURE ONLY.

Imported only by tests/ (and tools that check the engine); never by neuralstyletransferv1_amd/.  Restates the
reference's arithmetic with the same torch-CPU fp32 ops the reference uses:
  masks_from_geometry   the pattern generators (region_blend.py:109-516) given the random draws
  feather               gaussian_blur_mask / feather_mask (region_blend.py:69-102): reflect pad + conv2d
  composite_adv         composite_regions / composite_regions_advanced (region_blend.py:1049-1108, 1589-1679)
  composite_crops       composite_from_crops incl. place_crop and the coverage-gap fill (region_blend.py:2080-2294)
  rotate                rotate_all_masks (region_blend.py:25-66): cv2.getRotationMatrix2D + cv2.warpAffine
                        (INTER_LINEAR, BORDER_REPLICATE) restated in numpy after OpenCV's fixed-point warp --
                        cv2 is absent here, so this stage is PARITY UNPINNED.
The random draws (mode pick, points, centres, wave parameters, quad splits) come from the engine's host
restatement neuralstyletransferv1_amd.regions.draw_geometry; both are pinned bit-exact against masks made by
the reference module itself (tests/golden/regions.npz, made by tests/golden/make_golden_regions.py).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F


def masks_from_geometry(g, H: int, W: int) -> torch.Tensor:
    """Hard masks [count,H,W] fp32, region_blend.py's tensor expressions verbatim in meaning."""
    out = []
    yy = torch.arange(H, dtype=torch.float32).view(H, 1).expand(H, W)
    xx = torch.arange(W, dtype=torch.float32).view(1, W).expand(H, W)
    if g.kind == "rects":  # grid_masks :120-133, fractal_quad_masks :359-362
        for (y1, y2, x1, x2) in g.rects:
            m = torch.zeros(H, W)
            m[y1:y2, x1:x2] = 1.0
            out.append(m)
    elif g.kind == "voronoi":  # :198-234
        d = []
        for k, (px, py) in enumerate(g.points):
            dist = torch.sqrt((xx - px) ** 2 + (yy - py) ** 2)
            d.append(dist / g.divisor[k] if g.divisor[k] != 0 else dist)
        nearest = torch.stack(d, 0).argmin(dim=0)
        out = [(nearest == k).float() for k in range(len(g.points))]
    else:
        if g.kind == "diagonal":  # :150-162
            t = xx + yy if g.ivals[0] else (W - 1 - xx) + yy
            t = t / t.max()
        elif g.kind == "radial":  # :384-389
            cx, cy = g.ivals[0], g.ivals[1]
            t = (torch.atan2(yy - cy, xx - cx) + math.pi + g.dvals[0]) % (2 * math.pi)
        elif g.kind == "waves":  # :419-437
            freq, amp, phase = g.dvals[0], g.dvals[1], g.dvals[2]
            yc, xc = yy / H, xx / W
            if g.ivals[0] == 0:
                t = yc + torch.sin(xc * freq * 2 * math.pi + phase) * amp
            elif g.ivals[0] == 1:
                t = xc + torch.sin(yc * freq * 2 * math.pi + phase) * amp
            else:
                dg = (xc + yc) / 2
                t = dg + torch.sin(dg * freq * 2 * math.pi + phase) * amp
            t = (t - t.min()) / (t.max() - t.min() + 1e-6)
        elif g.kind == "spiral":  # :466-475
            yc, xc = yy - g.ivals[1], xx - g.ivals[0]
            r = torch.sqrt(xc ** 2 + yc ** 2)
            theta = torch.atan2(yc, xc) + math.pi + g.dvals[1]
            t = (theta + r / int(g.dvals[2]) * g.dvals[0] * 2 * math.pi) % (2 * math.pi)
            t = t / (2 * math.pi)
        else:  # concentric :501-506
            yc, xc = yy - g.ivals[1], xx - g.ivals[0]
            r = torch.sqrt(xc ** 2 + yc ** 2)
            t = r / r.max()
        out = [((t >= g.lo[k]) & (t < g.hi[k])).float() for k in range(g.n_gen)]
    while len(out) < g.count:  # :977-978
        out.append(out[-1].clone() if out else torch.ones(H, W))
    return torch.stack(out[:g.count], 0)


def feather(masks: torch.Tensor, feather_px: int) -> torch.Tensor:
    """feather_mask of each plane (region_blend.py:69-102)."""
    if feather_px <= 0:
        return masks
    sigma = feather_px / 3.0
    ks = int(6 * sigma + 1)
    if ks % 2 == 0:
        ks += 1
    ks = max(3, ks)
    x = torch.arange(ks, dtype=torch.float32) - ks // 2
    k1 = torch.exp(-x ** 2 / (2 * sigma ** 2))
    k1 = k1 / k1.sum()
    k2 = (k1.view(-1, 1) @ k1.view(1, -1)).view(1, 1, ks, ks)
    pad = ks // 2
    return torch.cat([F.conv2d(F.pad(m[None, None], (pad, pad, pad, pad), mode="reflect"), k2)[0]
                      for m in masks], 0)


def composite_adv(outputs_by_scale: Dict[float, List[torch.Tensor]], masks: torch.Tensor, configs,
                  original: Optional[torch.Tensor], H: int, W: int) -> torch.Tensor:
    """composite_regions_advanced (region_blend.py:1589-1679); with one model per region at weight 1 this is
    composite_regions (:1049-1108) exactly.  outputs [3,H',W'] in [0,1], original [3,H,W] or None."""
    result = torch.zeros(1, 3, H, W)
    wsum = torch.zeros(1, 1, H, W)
    if original is not None:
        original = original.unsqueeze(0)
    for k, cfg in enumerate(configs):
        m = masks[k].view(1, 1, H, W)
        scale = cfg.scale
        if scale not in outputs_by_scale:
            scale = min(list(outputs_by_scale.keys()), key=lambda s: abs(s - cfg.scale))
        rb = torch.zeros(1, 3, H, W)
        for mi, w in zip(cfg.model_indices, cfg.model_weights):
            if mi == -1:
                src = original
            else:
                src = outputs_by_scale[scale][mi].unsqueeze(0)
                if src.shape[-2:] != (H, W):
                    src = F.interpolate(src, size=(H, W), mode="bilinear", align_corners=False)
            rb += w * src
        result += rb * m.expand(1, 3, H, W)
        wsum += m
    return (result / wsum.expand(1, 3, H, W).clamp(min=1e-6)).squeeze(0).clamp(0, 1)


def composite_crops(styled: Dict[int, Dict[int, torch.Tensor]], boxes: Sequence, configs, masks: torch.Tensor,
                    original: Optional[torch.Tensor], H: int, W: int, weights_per_region=None) -> torch.Tensor:
    """composite_from_crops (region_blend.py:2186-2294): styled[model][region] = decoded crop [3,h,w]."""
    canvas = torch.zeros(3, H, W)
    wsum = torch.zeros(1, H, W)
    for k, ((x1, y1, x2, y2), cfg) in enumerate(zip(boxes, configs)):
        ch, cw = y2 - y1, x2 - x1
        wts = weights_per_region[k] if weights_per_region is not None else cfg.model_weights
        rb = torch.zeros(3, ch, cw)
        for mi, w in zip(cfg.model_indices, wts):
            src = original[:, y1:y2, x1:x2].clone() if mi == -1 else styled[mi][k]
            if src.shape[1] != ch or src.shape[2] != cw:
                src = F.interpolate(src.unsqueeze(0), size=(ch, cw), mode="bilinear", align_corners=False).squeeze(0)
            rb += w * src
        cm = masks[k, y1:y2, x1:x2].view(1, 1, ch, cw)
        canvas[:, y1:y2, x1:x2] += rb * cm.squeeze(0).expand(3, -1, -1)
        wsum[:, y1:y2, x1:x2] += cm.squeeze(0)
    gap = (wsum < 0.1).float()
    if gap.sum() > 0:
        gap3 = gap.expand(3, -1, -1)
        if original is not None:
            canvas = canvas + original * gap3
            wsum = wsum + gap
        else:
            for ks in (5, 11, 21):
                p = ks // 2
                cd = F.max_pool2d(canvas.unsqueeze(0), kernel_size=ks, stride=1, padding=p).squeeze(0)
                wd = F.max_pool2d(wsum.unsqueeze(0), kernel_size=ks, stride=1, padding=p).squeeze(0)
                canvas = canvas * (1 - gap3) + cd * gap3
                wsum = wsum * (1 - gap) + wd * gap
                gap = (wsum < 0.1).float()
                gap3 = gap.expand(3, -1, -1)
                if gap.sum() == 0:
                    break
    return (canvas / wsum.expand(3, -1, -1).clamp(min=1e-6)).clamp(0, 1)


def bbox(mask: torch.Tensor, threshold: float = 0.01):
    """compute_mask_bbox (region_blend.py:1969-1994) -> (x1, y1, x2, y2)."""
    H, W = mask.shape
    m = mask.numpy()
    rows, cols = np.any(m > threshold, axis=1), np.any(m > threshold, axis=0)
    if not rows.any() or not cols.any():
        return (0, 0, W, H)
    y1, y2 = np.where(rows)[0][[0, -1]]
    x1, x2 = np.where(cols)[0][[0, -1]]
    return (int(x1), int(y1), int(x2) + 1, int(y2) + 1)


def _warp_affine_replicate(src: np.ndarray, M: np.ndarray) -> np.ndarray:
    """cv2.warpAffine(src f32, M, (W,H), INTER_LINEAR, BORDER_REPLICATE) after OpenCV's imgwarp: inverse map in
    1/1024 fixed point (per-column cvRound(M00*x*1024), per-row bases + 16), 1/32-pixel taps from the
    32x32 float weight table, taps clamped (PARITY UNPINNED: cv2 absent)."""
    H, W = src.shape
    D = M[0, 0] * M[1, 1] - M[0, 1] * M[1, 0]
    D = 1.0 / D if D != 0 else 0.0
    A11, A22, A12, A21 = M[1, 1] * D, M[0, 0] * D, -M[0, 1] * D, -M[1, 0] * D
    b1 = -A11 * M[0, 2] - A12 * M[1, 2]
    b2 = -A21 * M[0, 2] - A22 * M[1, 2]
    xs = np.arange(W, dtype=np.float64)
    adelta = np.rint(A11 * xs * 1024.0).astype(np.int64)
    bdelta = np.rint(A21 * xs * 1024.0).astype(np.int64)
    out = np.empty_like(src)
    for y in range(H):
        X0 = int(np.rint((A12 * y + b1) * 1024.0)) + 16
        Y0 = int(np.rint((A22 * y + b2) * 1024.0)) + 16
        X = (X0 + adelta) >> 5
        Y = (Y0 + bdelta) >> 5
        sx, sy = X >> 5, Y >> 5
        fx = (X & 31).astype(np.float32) * np.float32(1 / 32)
        fy = (Y & 31).astype(np.float32) * np.float32(1 / 32)
        one = np.float32(1)
        w00, w01, w10, w11 = (one - fy) * (one - fx), (one - fy) * fx, fy * (one - fx), fy * fx
        x0, x1 = np.clip(sx, 0, W - 1), np.clip(sx + 1, 0, W - 1)
        y0, y1 = np.clip(sy, 0, H - 1), np.clip(sy + 1, 0, H - 1)
        t0 = src[y0, x0] * w00 + src[y0, x1] * w01
        t1 = src[y1, x0] * w10 + src[y1, x1] * w11
        out[y] = t0 + t1
    return out


def rotate(masks: torch.Tensor, angle_deg: float) -> torch.Tensor:
    """rotate_all_masks (region_blend.py:49-66) with cv2.getRotationMatrix2D((W/2, H/2), angle, 1.0)."""
    if angle_deg == 0:
        return masks
    K, H, W = masks.shape
    a = angle_deg * (math.pi / 180.0)  # cv2: angle *= CV_PI/180
    al, be = math.cos(a), math.sin(a)
    cx, cy = W / 2.0, H / 2.0
    M = np.array([[al, be, (1 - al) * cx - be * cy], [-be, al, be * cx + (1 - al) * cy]])
    rot = [torch.from_numpy(_warp_affine_replicate(masks[k].numpy(), M)) for k in range(K)]
    s = torch.zeros(H, W)
    for r in rot:
        s += r
    s = s.clamp(min=1e-6)
    return torch.stack([r / s for r in rot], 0)


# ------------------------------------------------------------------ --region_morph (region_blend.py:535-810)
def simplex_noise(H: int, W: int, frequency: float, octaves: int, seed: int, time_offset: float = 0.0) -> np.ndarray:
    """_simplex_noise_2d (region_blend.py:604-652): float64 octave sums into a float32 accumulator,
    normalised to [0, 1] in float32 (pinned by tests/golden/regions.npz flow_*)."""
    rng = np.random.default_rng(seed)
    xx, yy = np.meshgrid(np.linspace(0, frequency, W), np.linspace(0, frequency, H))
    acc = np.zeros((H, W), dtype=np.float32)
    amp, total, fm = 1.0, 0.0, 1.0
    for o in range(octaves):
        ox = time_offset * (0.5 + 0.3 * o) + rng.random() * 1000
        oy = time_offset * (0.3 + 0.2 * o) + rng.random() * 1000
        nz = np.sin(xx * fm + ox) * np.cos(yy * fm + oy)
        nz += np.sin((xx + yy) * fm * 0.7 + ox * 0.8) * 0.5
        nz += np.cos((xx - yy) * fm * 0.5 + oy * 0.6) * 0.3
        acc += nz * amp
        total += amp
        amp *= 0.5
        fm *= 2.0
    acc = acc / total
    return (acc - acc.min()) / (acc.max() - acc.min() + 1e-6)


def flow_field(H: int, W: int, frequency: float, seed: int, t: float):
    """_generate_flow_field (region_blend.py:655-667)."""
    return (simplex_noise(H, W, frequency, 2, seed, t) * 2 - 1,
            simplex_noise(H, W, frequency, 2, seed + 1000, t * 1.3) * 2 - 1)


def _remap_reflect(src: np.ndarray, map_x: np.ndarray, map_y: np.ndarray) -> np.ndarray:
    """cv2.remap(src f32, map_x, map_y, INTER_LINEAR, BORDER_REFLECT) after OpenCV: cvRound(map * 32) fixed point,
    float weight table, each tap reflected (fedcba|abcdef) -- PARITY UNPINNED (cv2 absent)."""
    H, W = src.shape
    X = np.rint(map_x.astype(np.float32) * np.float32(32)).astype(np.int64)
    Y = np.rint(map_y.astype(np.float32) * np.float32(32)).astype(np.int64)
    sx, sy = X >> 5, Y >> 5
    fx = (X & 31).astype(np.float32) * np.float32(1 / 32)
    fy = (Y & 31).astype(np.float32) * np.float32(1 / 32)

    def refl(p, n):
        if n == 1:
            return np.zeros_like(p)
        p = p.copy()
        for _ in range(4):
            p = np.where(p < 0, -p - 1, p)
            p = np.where(p >= n, 2 * n - p - 1, p)
        return p
    x0, x1, y0, y1 = refl(sx, W), refl(sx + 1, W), refl(sy, H), refl(sy + 1, H)
    one = np.float32(1)
    t0 = src[y0, x0] * ((one - fy) * (one - fx)) + src[y0, x1] * ((one - fy) * fx)
    t1 = src[y1, x0] * (fy * (one - fx)) + src[y1, x1] * (fy * fx)
    return (t0 + t1).astype(np.float32)


def morph(masks: torch.Tensor, mode: str, speed: float, amplitude: float, frequency: float, seed: int,
          frame_idx: int) -> torch.Tensor:
    """warp_all_masks_organic (region_blend.py:737-810) with warp_mask_organic (:670-734) per plane."""
    K, H, W = masks.shape
    t = frame_idx * speed * 0.02
    warped = []
    for j in range(K):
        sd = seed + j * 100
        if mode == "tentacle":
            fx, fy = flow_field(H, W, frequency * 2, sd, t)
            fy += np.sin(np.linspace(0, 1, H)[:, None] * np.pi * 3 + t) * 0.5
        elif mode == "wave":
            fx = np.sin(np.linspace(0, np.pi * frequency, H)[:, None] + t * 2) * np.ones((H, W))
            fy = np.cos(np.linspace(0, np.pi * frequency, W)[None, :] + t * 1.5) * np.ones((H, W))
        elif mode == "pulse":
            yc, xc = np.arange(H)[:, None] - H // 2, np.arange(W)[None, :] - W // 2
            r = np.sqrt(xc ** 2 + yc ** 2) + 1e-6
            th = np.arctan2(yc, xc)
            pu = np.sin(r * 0.05 - t * 3) * 0.5 + 0.5
            fx, fy = np.cos(th) * pu, np.sin(th) * pu
        else:
            fx, fy = flow_field(H, W, frequency, sd, t)
        md = max(H, W) * amplitude
        fx, fy = fx * md, fy * md
        gy = np.arange(H, dtype=np.float32)[:, None].repeat(W, axis=1)
        gx = np.arange(W, dtype=np.float32)[None, :].repeat(H, axis=0)
        warped.append(torch.from_numpy(_remap_reflect(masks[j].numpy(), (gx + fx).astype(np.float32),
                                                      (gy + fy).astype(np.float32))))
    s = torch.zeros(H, W)
    for m in warped:
        s += m
    gap = (s < 0.1).float()
    if gap.sum() > 0:
        filled = list(warped)
        for ks in (5, 11, 21, 41):
            nf = [m * (1 - gap) + F.max_pool2d(m[None, None], ks, 1, ks // 2)[0, 0] * gap for m in filled]
            s = torch.zeros(H, W)
            for m in nf:
                s += m
            gap = (s < 0.1).float()
            filled = nf
            if gap.sum() == 0:
                break
        warped = filled
    s = s.clamp(min=1e-6)
    return torch.stack([m / s for m in warped], 0)
