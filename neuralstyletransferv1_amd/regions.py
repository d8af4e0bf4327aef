"""Region-blend compositor on the MI355X engine.

Drop-in for the reference's region_blend.py as pipeline.py drives it:
  * --region_mode (standard path, pipeline.py:1720-1839): every model styles the whole frame, then
    blend_by_regions / blend_by_regions_advanced (region_blend.py:1690-1787, 1832-1951) composite them
    through soft region masks;
  * --region_optimize (pipeline.py:1120-1407): each region's padded bounding box is cropped, styled only
    by the models that region uses, and composite_from_crops (region_blend.py:2186-2294) reassembles it.

Split of the work:
  host (this module) -- the reference's control logic, restated: random.Random draws in the reference's
      order (so a seed gives the reference's regions and assignments), blend / scale / morph / animation
      spec parsing, model assignment, crop planning;
  GPU (libnst_hip.so, include/nst_hip.h "Region-blend compositor") -- mask rendering, Gaussian feather,
      rotation, bounding boxes, crop inputs, low-resolution sources and both composites (ToPILImage
      truncation fused).  No CPU fallback.

--region_morph's organic warp (region_blend.py:535-810) runs on the GPU too: the noise fields' numpy PCG64
draws are made here in the reference's order, the fields, cv2.remap (restated: cv2 is absent, parity
unpinned), the gap dilations and the renormalisation in region_ops.hip.
"""
from __future__ import annotations

import ctypes
import math
import random
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib
from ._lib import NstError, check, lib

MODES = ("grid", "diagonal", "voronoi", "fractal", "radial", "waves", "spiral", "concentric", "random")
MORPH_MODES = ("blob", "tentacle", "wave", "pulse")
_MODEL_LETTERS = {"A": 0, "B": 1, "C": 2, "D": 3, "E": 4, "F": 5, "G": 6, "H": 7, "O": -1, "ORIGINAL": -1}
_OFF = ("none", "static", "off", "0")


# ============================================================================ specs and animations
@dataclass
class RegionConfig:
    """region_blend.py:1116-1120: models blended in a region (-1 = original), weights, scale."""
    model_indices: List[int]
    model_weights: List[float]
    scale: float


@dataclass
class BlendAnimation:
    """region_blend.py:1184-1192."""
    enabled: bool = False
    period: float = 120.0
    min_opacity: float = 0.0
    max_opacity: float = 1.0
    phase_offset: float = 0.0
    waveform: str = "sine"
    per_model_phase: bool = True


@dataclass
class ScaleAnimation:
    """region_blend.py:1334-1341."""
    enabled: bool = False
    period: float = 60.0
    min_scale: float = 0.5
    max_scale: float = 1.0
    phase_offset: float = 0.0
    waveform: str = "sine"


@dataclass
class MorphAnimation:
    """region_blend.py:524-532."""
    enabled: bool = False
    speed: float = 1.0
    amplitude: float = 0.15
    frequency: float = 3.0
    octaves: int = 3
    mode: str = "blob"
    seed: int = 42


_WAVEFORMS = {
    "sine": lambda t: (math.sin(2 * math.pi * t) + 1) / 2,
    "triangle": lambda t: t * 2 if t < 0.5 else 2 - (t * 2),
    "sawtooth": lambda t: t,
    "sawtooth_down": lambda t: 1 - t,
    "square": lambda t: 1.0 if t < 0.5 else 0.0,
}


def compute_harmonic_value(frame_idx: int, period: float, min_val: float = 0.0, max_val: float = 1.0,
                           phase_offset: float = 0.0, waveform: str = "sine") -> float:
    """region_blend.py:1127-1180: position in the cycle (phase in degrees) -> waveform -> [min, max]
    (unknown waveforms are sine; a non-positive period gives the midpoint)."""
    if period <= 0:
        return (min_val + max_val) / 2
    t = ((frame_idx / period) + (phase_offset / 360.0)) % 1.0
    wave = _WAVEFORMS.get(waveform, _WAVEFORMS["sine"])(t)
    return min_val + wave * (max_val - min_val)


def compute_animated_weights(base_weights: List[float], frame_idx: int, anim: BlendAnimation) -> List[float]:
    """region_blend.py:1195-1247: each model's weight oscillates (phase step 360/n), renormalised."""
    n = len(base_weights)
    if not anim.enabled or n <= 1:
        return base_weights
    raw = []
    for i, bw in enumerate(base_weights):
        phase = anim.phase_offset + (i * 360.0 / n if anim.per_model_phase else 0.0)
        raw.append(compute_harmonic_value(frame_idx, anim.period, anim.min_opacity, anim.max_opacity, phase,
                                          anim.waveform) * bw)
    total = sum(raw)
    return [1.0 / n] * n if total < 1e-6 else [r / total for r in raw]


def compute_animated_scale(base_scale: float, frame_idx: int, anim: ScaleAnimation) -> float:
    """region_blend.py:1344-1370."""
    if not anim.enabled:
        return base_scale
    return compute_harmonic_value(frame_idx, anim.period, anim.min_scale, anim.max_scale, anim.phase_offset,
                                  anim.waveform)


def _spec_fields(spec: Optional[str]):
    """'period,waveform,phase,min,max' -> (period, waveform, phase, [min, max] strings) or None if off."""
    if not spec or spec.lower() in _OFF:
        return None
    parts = spec.split(",")
    try:
        period = float(parts[0].strip())
    except ValueError:
        return None
    rest = [p.strip() for p in parts[1:]]
    return period, rest


def parse_blend_animation(spec: Optional[str]) -> BlendAnimation:
    """region_blend.py:1250-1290 (defaults: sine, phase 0, opacity 0..1)."""
    f = _spec_fields(spec)
    if f is None:
        return BlendAnimation(enabled=False)
    period, rest = f
    get = lambda i, d: rest[i] if len(rest) > i else d  # noqa: E731
    return BlendAnimation(enabled=True, period=period, waveform=get(0, "sine"), phase_offset=float(get(1, 0.0)),
                          min_opacity=float(get(2, 0.0)), max_opacity=float(get(3, 1.0)), per_model_phase=True)


def parse_scale_animation(spec: Optional[str]) -> ScaleAnimation:
    """region_blend.py:1373-1412 (defaults: sine, phase 0, scale 0.5..1)."""
    f = _spec_fields(spec)
    if f is None:
        return ScaleAnimation(enabled=False)
    period, rest = f
    get = lambda i, d: rest[i] if len(rest) > i else d  # noqa: E731
    return ScaleAnimation(enabled=True, period=period, waveform=get(0, "sine"), phase_offset=float(get(1, 0.0)),
                          min_scale=float(get(2, 0.5)), max_scale=float(get(3, 1.0)))


def _per_region(spec: Optional[str], n: int, parse, off):
    """'spec|spec|...' cycles over the regions; a spec without '|' applies to all (region_blend.py:1293-1326)."""
    if not spec:
        return [off] * n
    if "|" not in spec:
        return [parse(spec)] * n
    parts = spec.split("|")
    return [parse(parts[i % len(parts)].strip()) for i in range(n)]


def parse_region_blend_animations(spec: Optional[str], num_regions: int) -> List[BlendAnimation]:
    return _per_region(spec, num_regions, parse_blend_animation, BlendAnimation(enabled=False))


def parse_region_scale_animations(spec: Optional[str], num_regions: int) -> List[ScaleAnimation]:
    return _per_region(spec, num_regions, parse_scale_animation, ScaleAnimation(enabled=False))


def parse_morph_animation(spec: Optional[str]) -> MorphAnimation:
    """region_blend.py:813-872: 'mode' | 'speed[,amplitude[,frequency[,mode]]]'; unparsable numbers make the
    whole spec a mode name."""
    if not spec or spec.lower() in ("none", "off", "0", "static"):
        return MorphAnimation(enabled=False)
    if spec.lower() in MORPH_MODES:
        return MorphAnimation(enabled=True, mode=spec.lower())
    parts = [p.strip() for p in spec.split(",")]
    keys = ("speed", "amplitude", "frequency")
    try:
        kw = {k: float(v) for k, v in zip(keys, parts[:3])}
    except ValueError:
        return MorphAnimation(enabled=True, mode=spec.lower())
    if len(parts) >= 4:
        kw["mode"] = parts[3].lower()
    return MorphAnimation(enabled=True, **kw)


def parse_region_sizes(spec: Optional[str], num_regions: int) -> Optional[List[float]]:
    """region_blend.py:885-922: relative voronoi cell sizes, cycled or truncated to num_regions."""
    if not spec:
        return None
    try:
        vals = [float(p) for p in (q.strip() for q in spec.replace("|", ",").split(",")) if p]
    except ValueError:
        return None
    if len(vals) < num_regions:
        return [vals[i % len(vals)] for i in range(num_regions)]
    return vals[:num_regions]


def parse_region_seed(seed_str: Optional[str], optimized: bool, animating: bool) -> Optional[int]:
    """Seed rules of the two paths: --region_optimize defaults to 42 and falls back to 42 on garbage
    (pipeline.py:1150-1161); the standard path defaults to 42 only while rotating/morphing and to a fresh
    random draw on garbage (:1740-1754)."""
    if seed_str is None:
        return 42 if (optimized or animating) else None
    s = str(seed_str).lower()
    if s == "random":
        return None
    if s == "fixed":
        return 42
    try:
        return int(seed_str)
    except ValueError:
        return 42 if optimized else None


def _rng(seed: Optional[int]) -> random.Random:
    return random.Random(seed) if seed is not None else random.Random()


def assign_models_to_regions(num_regions: int, num_models: int, assignment: str = "random",
                             weights: Optional[List[float]] = None, seed: Optional[int] = None,
                             original_chance: float = 0.0) -> List[int]:
    """region_blend.py:983-1046 (-1 = the original frame)."""
    rng = _rng(seed)
    with_orig = original_chance > 0
    if assignment == "sequential":
        pool = list(range(num_models)) + ([-1] if with_orig else [])
        return [pool[i % len(pool)] for i in range(num_regions)]
    if assignment == "random":
        out = []
        for _ in range(num_regions):
            # the draw for the original happens only when original_chance > 0 (short-circuit)
            out.append(-1 if (with_orig and rng.random() < original_chance) else rng.randint(0, num_models - 1))
        return out
    if assignment == "weighted":
        w = list(weights) if weights is not None else [1.0 / num_models] * num_models
        total = sum(w[:num_models])
        if with_orig:
            probs = [(x / total) * (1.0 - original_chance) for x in w[:num_models]] + [original_chance]
            return rng.choices(list(range(num_models)) + [-1], weights=probs, k=num_regions)
        return rng.choices(range(num_models), weights=[x / total for x in w[:num_models]], k=num_regions)
    raise ValueError(f"Unknown assignment mode: {assignment}")


def _parse_blend_spec(spec: str, num_regions: int, num_models: int, scales: List[float]) -> List[RegionConfig]:
    """region_blend.py:1510-1586: 'A+B|C:0.7+D:0.3|O' -> per-region model lists; unspecified weights share
    what the explicit ones leave, then every region's weights are normalised."""
    per_region = [s.strip() for s in spec.upper().split("|") if s.strip()]
    configs = []
    for i in range(num_regions):
        idx, wts = [], []
        for part in (p.strip() for p in per_region[i % len(per_region)].split("+")):
            if not part:
                continue
            name, _, wstr = part.partition(":")
            name = name.strip()
            if name in _MODEL_LETTERS:
                idx.append(_MODEL_LETTERS[name])
            elif name.isdigit():
                idx.append(int(name))
            else:
                raise ValueError(f"Unknown model in blend spec: {name}")
            wts.append(float(wstr.strip()) if ":" in part else None)
        unset = wts.count(None)
        if unset:
            share = max(0.0, 1.0 - sum(x for x in wts if x is not None)) / unset
            wts = [share if x is None else x for x in wts]
        total = sum(wts)
        wts = [x / total for x in wts] if total > 0 else [1.0 / len(idx)] * len(idx)
        configs.append(RegionConfig(idx, wts, scales[i % len(scales)] if scales else 1.0))
    return configs


def _parse_scales(scale_spec: Optional[str]) -> List[float]:
    if not scale_spec:
        return []
    return [float(s.strip()) for s in scale_spec.replace(",", "|").split("|") if s.strip()]


def parse_region_configs(num_regions: int, num_models: int, assignment: str = "sequential",
                         blend_spec: Optional[str] = None, scale_spec: Optional[str] = None,
                         seed: Optional[int] = None, original_chance: float = 0.0) -> List[RegionConfig]:
    """region_blend.py:1451-1507 (assignment weights are not passed on here, as in the reference)."""
    scales = _parse_scales(scale_spec)
    if blend_spec:
        return _parse_blend_spec(blend_spec, num_regions, num_models, scales)
    picks = assign_models_to_regions(num_regions, num_models, assignment, None, seed, original_chance)
    return [RegionConfig([m], [1.0], scales[i % len(scales)] if scales else 1.0) for i, m in enumerate(picks)]


def get_required_scales(num_regions: int, num_models: int, assignment: str = "sequential",
                        blend_spec: Optional[str] = None, scale_spec: Optional[str] = None,
                        seed: Optional[int] = None, original_chance: float = 0.0) -> List[float]:
    """region_blend.py:1796-1829 (set order kept: it decides ties of the nearest-scale fallback)."""
    scales = _parse_scales(scale_spec)
    if not scales:
        return [1.0]
    if blend_spec:
        return list(set(c.scale for c in _parse_blend_spec(blend_spec, num_regions, num_models, scales)))
    return list(set(scales))


# ============================================================================ mask geometry
@dataclass
class Geometry:
    """One generate_region_masks call, reduced to what the mask kernel needs (include/nst_hip.h NST_RG_*)."""
    mode: str                 # the generator actually used ('random' resolved)
    kind: str                 # _lib.RG_KINDS key
    count: int
    n_gen: int
    ivals: Tuple[int, int, int] = (0, 0, 0)
    dvals: Tuple[float, float, float, float] = (0.0, 0.0, 0.0, 0.0)
    lo: Tuple[float, ...] = ()
    hi: Tuple[float, ...] = ()
    rects: Tuple[Tuple[int, int, int, int], ...] = ()
    points: Tuple[Tuple[float, float], ...] = ()
    divisor: Tuple[float, ...] = ()


def _bands(count: int) -> Tuple[Tuple[float, ...], Tuple[float, ...]]:
    return tuple(i / count for i in range(count)), tuple((i + 1) / count for i in range(count))


def _balanced_points(W: int, H: int, count: int, rng: random.Random, jitter: float = 0.3):
    """region_blend.py:239-304: one jittered point per cell of a ~aspect-matched grid, shuffled."""
    aspect = W / H
    cols = max(1, int(math.sqrt(count * aspect) + 0.5))
    rows = max(1, int(math.sqrt(count / aspect) + 0.5))
    while cols * rows < count:
        if cols / rows < aspect:
            cols += 1
        else:
            rows += 1
    cw, ch = W / cols, H / rows
    pts = []
    for r in range(rows):
        for c in range(cols):
            if len(pts) >= count:
                break
            jx = (rng.random() - 0.5) * cw * jitter
            jy = (rng.random() - 0.5) * ch * jitter
            pts.append((max(0, min(W - 1, (c + 0.5) * cw + jx)), max(0, min(H - 1, (r + 0.5) * ch + jy))))
    while len(pts) < count:
        pts.append((rng.randint(0, W - 1), rng.randint(0, H - 1)))
    rng.shuffle(pts)
    return pts[:count]


def _fractal_rects(H: int, W: int, count: int, rng: random.Random, max_depth: int = 4):
    """region_blend.py:307-355: random quad-tree leaves (y1, y2, x1, x2), depth-first in shuffled order."""
    leaves = []

    def visit(y1, y2, x1, x2, depth):
        if len(leaves) >= count:
            return
        if depth >= max_depth or (y2 - y1) < 20 or (x2 - x1) < 20:
            leaves.append((y1, y2, x1, x2))
            return
        if rng.random() > 0.4 and depth > 0:
            leaves.append((y1, y2, x1, x2))
            return
        my = (y1 + y2) // 2 + rng.randint(-10, 10)
        mx = (x1 + x2) // 2 + rng.randint(-10, 10)
        my = max(y1 + 10, min(y2 - 10, my))
        mx = max(x1 + 10, min(x2 - 10, mx))
        quads = [(y1, my, x1, mx), (y1, my, mx, x2), (my, y2, x1, mx), (my, y2, mx, x2)]
        rng.shuffle(quads)
        for q in quads:
            if len(leaves) >= count:
                break
            visit(*q, depth + 1)

    visit(0, H, 0, W, 0)
    return leaves[:count]


def _corner_rmax(H: int, W: int, cx: int, cy: int) -> float:
    """r.max() of sqrt((x-cx)^2 + (y-cy)^2) over the frame in float32 (attained at a corner)."""
    best = np.float32(0)
    for x in (0, W - 1):
        for y in (0, H - 1):
            dx, dy = np.float32(x) - np.float32(cx), np.float32(y) - np.float32(cy)
            best = max(best, np.sqrt(dx * dx + dy * dy, dtype=np.float32))
    return float(best)


def draw_geometry(H: int, W: int, mode: str, count: int, seed: Optional[int] = None,
                  region_sizes: Optional[List[float]] = None) -> Geometry:
    """The random draws of generate_region_masks (region_blend.py:925-980) in the reference's order."""
    rng = _rng(seed)
    if mode == "random":
        mode = rng.choice([m for m in MODES if m != "random"])
        print(f"[region] Randomly selected mode: {mode}")
    if mode not in MODES:
        raise ValueError(f"Unknown region mode: {mode}. Available: {list(MODES)}")
    if region_sizes and mode != "voronoi":
        print(f"[region] Warning: --region_sizes only works with voronoi mode, ignoring for {mode}")
    lo, hi = _bands(count)
    if mode == "grid":  # region_blend.py:109-135
        g = int(math.ceil(math.sqrt(count)))
        chh, cww = H / g, W / g
        rects = []
        for i in range(count):
            r, c = divmod(i, g)
            rects.append((int(r * chh), min(int((r + 1) * chh), H), int(c * cww), min(int((c + 1) * cww), W)))
        return Geometry(mode, "rects", count, count, rects=tuple(rects))
    if mode == "fractal":
        rects = _fractal_rects(H, W, count, rng)
        return Geometry(mode, "rects", count, len(rects), rects=tuple(rects))
    if mode == "diagonal":  # region_blend.py:154-162
        tl = rng.random() > 0.5
        return Geometry(mode, "diagonal", count, count, ivals=(1 if tl else 0, 0, 0),
                        dvals=(0.0, 0.0, 0.0, float((W - 1) + (H - 1))), lo=lo, hi=hi)
    if mode == "voronoi":  # region_blend.py:195-228
        pts = _balanced_points(W, H, count, rng)
        if region_sizes:
            total = sum(region_sizes)
            nw = [x * count / total for x in region_sizes]
            div = tuple(math.sqrt(nw[i] if i < len(nw) else 1.0) + 1e-6 for i in range(count))
        else:
            div = (0.0,) * count
        return Geometry(mode, "voronoi", count, count, points=tuple((float(x), float(y)) for x, y in pts), divisor=div)
    if mode == "radial":  # region_blend.py:377-399
        cx = W // 2 + rng.randint(-W // 4, W // 4)
        cy = H // 2 + rng.randint(-H // 4, H // 4)
        rot = rng.random() * 2 * math.pi
        wedge = 2 * math.pi / count
        return Geometry(mode, "radial", count, count, ivals=(cx, cy, 0), dvals=(rot, 0.0, 0.0, 0.0),
                        lo=tuple(i * wedge for i in range(count)), hi=tuple((i + 1) * wedge for i in range(count)))
    if mode == "waves":  # region_blend.py:413-416
        freq = rng.uniform(1.5, 4.0)
        amp = rng.uniform(0.05, 0.15)
        direction = rng.choice(["horizontal", "vertical", "diagonal"])
        phase = rng.random() * 2 * math.pi
        return Geometry(mode, "waves", count, count, ivals=(("horizontal", "vertical", "diagonal").index(direction), 0, 0),
                        dvals=(freq, amp, phase, 0.0), lo=lo, hi=hi)
    if mode == "spiral":  # region_blend.py:459-463
        tight = rng.uniform(2.0, 5.0)
        rot = rng.random() * 2 * math.pi
        return Geometry(mode, "spiral", count, count, ivals=(W // 2, H // 2, 0), dvals=(tight, rot, float(max(H, W)), 0.0),
                        lo=lo, hi=hi)
    # concentric, region_blend.py:497-506
    cx = W // 2 + rng.randint(-W // 6, W // 6)
    cy = H // 2 + rng.randint(-H // 6, H // 6)
    return Geometry(mode, "concentric", count, count, ivals=(cx, cy, 0), dvals=(0.0, 0.0, 0.0, _corner_rmax(H, W, cx, cy)),
                    lo=lo, hi=hi)


def feather_taps(feather_px: int) -> Optional[np.ndarray]:
    """The 1-D taps of gaussian_blur_mask(sigma = feather/3) (region_blend.py:69-102) as the reference's torch
    arithmetic rounds them (fp32 exp, normalised by their fp32 sum); None when feather <= 0."""
    if feather_px <= 0:
        return None
    sigma = feather_px / 3.0
    ks = int(6 * sigma + 1)
    ks = max(3, ks + 1 if ks % 2 == 0 else ks)
    x = torch.arange(ks, dtype=torch.float32) - ks // 2
    k = torch.exp(-x ** 2 / (2 * sigma ** 2))
    return (k / k.sum()).numpy().astype(np.float32)


# ============================================================================ GPU side
def _arr(ctype, vals):
    vals = list(vals)
    return (ctype * max(1, len(vals)))(*vals)


def _stream(dev):
    return _lib.stream_ptr(dev)


def render_masks(geom: Geometry, H: int, W: int, feather: int, device) -> torch.Tensor:
    """generate_region_masks on the GPU: hard masks from `geom`, then feather_mask(feather) -> [K,H,W] f32."""
    dev = torch.device(device)
    K = geom.count
    if K > _lib.NST_REGION_MAX:
        raise NstError(f"{K} regions: the compositor takes at most {_lib.NST_REGION_MAX}")
    masks = torch.empty((K, H, W), dtype=torch.float32, device=dev)
    scratch = torch.empty((H * W + 2052 + 4,), dtype=torch.float32, device=dev) if geom.kind == "waves" else None
    rects = [v for r in geom.rects for v in r]
    pts = [v for p in geom.points for v in p]
    d = ctypes.c_double
    check(lib().nst_region_masks(_lib.RG_KINDS[geom.kind], K, geom.n_gen, _arr(ctypes.c_int, geom.ivals),
                                 _arr(d, geom.dvals), _arr(d, geom.lo), _arr(d, geom.hi), _arr(ctypes.c_int, rects),
                                 _arr(d, pts), _arr(d, geom.divisor), H, W, masks.data_ptr(),
                                 scratch.data_ptr() if scratch is not None else None, _stream(dev)), "nst_region_masks")
    return feather_planes(masks, feather)


def feather_planes(masks: torch.Tensor, feather: int) -> torch.Tensor:
    """feather_mask(m, feather) of every plane, in place (no-op for feather <= 0)."""
    taps = feather_taps(feather)
    if taps is None:
        return masks
    K, H, W = masks.shape
    scratch = torch.empty_like(masks)
    check(lib().nst_region_feather(masks.data_ptr(), K, H, W, taps.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                   len(taps), scratch.data_ptr(), _stream(masks.device)), "nst_region_feather")
    return masks


_MORPH_KIND = {"blob": 0, "tentacle": 1, "wave": 2, "pulse": 3}


def morph_offsets(morph: MorphAnimation, k: int) -> np.ndarray:
    """The random offsets of _simplex_noise_2d (region_blend.py:620-635) for warp_all_masks_organic's k planes:
    plane j seeds morph.seed + 100 j (field x) and that + 1000 (field y); per octave rng.random() * 1000 for x
    then y -> float64 [k][2][2][2]."""
    off = np.zeros((k, 2, 2, 2), dtype=np.float64)
    for j in range(k):
        for f, sd in enumerate((morph.seed + j * 100, morph.seed + j * 100 + 1000)):
            rng = np.random.default_rng(sd)
            for o in range(2):
                off[j, f, o, 0] = rng.random() * 1000
                off[j, f, o, 1] = rng.random() * 1000
    return off


def morph_planes(masks: torch.Tensor, morph: MorphAnimation, frame_idx: int) -> torch.Tensor:
    """warp_all_masks_organic (region_blend.py:737-810) -> new planes (the caller re-feathers them)."""
    if not morph.enabled:
        return masks
    K, H, W = masks.shape
    mode = _MORPH_KIND.get(morph.mode, 0)  # unknown modes take the blob branch (region_blend.py:714)
    freq = morph.frequency * 2 if mode == 1 else morph.frequency
    t = frame_idx * morph.speed * 0.02
    off = morph_offsets(morph, K) if mode <= 1 else np.zeros((K, 2, 2, 2))
    sz = ctypes.c_size_t()
    check(lib().nst_region_morph_scratch_floats(K, H, W, ctypes.byref(sz)), "nst_region_morph_scratch_floats")
    scratch = torch.empty((sz.value,), dtype=torch.float32, device=masks.device)
    out = torch.empty_like(masks)
    check(lib().nst_region_morph(masks.data_ptr(), K, H, W, mode, float(freq), float(t), float(max(H, W) * morph.amplitude),
                                 off.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), out.data_ptr(),
                                 scratch.data_ptr(), sz.value, _stream(masks.device)), "nst_region_morph")
    return out


def rotate_planes(masks: torch.Tensor, angle_deg: float) -> torch.Tensor:
    """rotate_all_masks (region_blend.py:49-66): warp + renormalise; the angle-0 call returns its input."""
    if angle_deg == 0:
        return masks
    K, H, W = masks.shape
    out = torch.empty_like(masks)
    check(lib().nst_region_rotate(masks.data_ptr(), K, H, W, float(angle_deg), out.data_ptr(), _stream(masks.device)),
          "nst_region_rotate")
    return out


def mask_bboxes(masks: torch.Tensor, threshold: float = 0.01) -> List[Tuple[int, int, int, int]]:
    """compute_mask_bbox of every plane (region_blend.py:1969-1994): (x1, y1, x2, y2); empty -> full frame."""
    K, H, W = masks.shape
    bb = torch.empty((K, 4), dtype=torch.int32, device=masks.device)
    check(lib().nst_region_bbox(masks.data_ptr(), K, H, W, float(np.float32(threshold)), bb.data_ptr(),
                                _stream(masks.device)), "nst_region_bbox")
    out = []
    for x1, y1, x2, y2 in bb.cpu().tolist():
        out.append((0, 0, W, H) if x2 < 0 else (x1, y1, x2, y2))
    return out


@dataclass
class Source:
    """One composite input: a raw model output (preset decode + bilinear fit on the fly) or a decoded image
    (preset 'none')."""
    y: torch.Tensor   # f32 NCHW [n,3,h,w]
    preset: str


def composite(sources: Sequence[Source], terms: Sequence[Sequence[Tuple[int, float]]], masks: torch.Tensor,
              orig_u8: Optional[torch.Tensor], boxes: Optional[Sequence[Tuple[int, int, int, int]]] = None,
              out_f32: bool = False) -> torch.Tensor:
    """Region composite of a batch (include/nst_hip.h nst_region_composite_u8). terms[k] = [(source, weight)]
    with source -1 for the original frame. Returns u8 NHWC [n,H,W,3] (or f32 NCHW [n,3,H,W] in [0,1])."""
    K, H, W = masks.shape
    if len(terms) != K:
        raise NstError(f"{len(terms)} region term lists for {K} masks")
    if len(sources) > _lib.NST_REGION_MAX_SRC:
        raise NstError(f"{len(sources)} sources: the compositor takes at most {_lib.NST_REGION_MAX_SRC}")
    dev = masks.device
    n = sources[0].y.shape[0] if sources else orig_u8.shape[0]
    for s in sources:
        _lib.require_gpu_tensor(s.y, "region source")
        if s.y.dtype != torch.float32 or not s.y.is_contiguous() or s.y.shape[0] != n or s.y.shape[1] != 3:
            raise NstError("region sources must be contiguous f32 [n,3,h,w]")
    if orig_u8 is not None and (orig_u8.dtype != torch.uint8 or tuple(orig_u8.shape) != (n, H, W, 3)
                                or not orig_u8.is_contiguous()):
        raise NstError("the original frames must be contiguous u8 [n,H,W,3]")
    T = _lib.NST_REGION_TERMS
    nt, ts, tw = [0] * K, [0] * (K * T), [0.0] * (K * T)
    for k, tl in enumerate(terms):
        if len(tl) > T:
            raise NstError(f"region {k} blends {len(tl)} sources (at most {T})")
        nt[k] = len(tl)
        for j, (s, w) in enumerate(tl):
            ts[k * T + j], tw[k * T + j] = int(s), float(np.float32(w))
    vp = ctypes.c_void_p
    ys = _arr(vp, [s.y.data_ptr() for s in sources])
    hw = _arr(ctypes.c_int, [v for s in sources for v in (s.y.shape[2], s.y.shape[3])])
    pr = _arr(ctypes.c_int, [_lib.PRESETS[s.preset] for s in sources])
    scratch, nfl = None, 0
    bx = None
    if boxes is not None:
        bx = _arr(ctypes.c_int, [v for b in boxes for v in b])
        sz = ctypes.c_size_t()
        check(lib().nst_region_scratch_floats(n, H, W, 1, int(orig_u8 is not None), ctypes.byref(sz)),
              "nst_region_scratch_floats")
        nfl = sz.value
        scratch = torch.empty((nfl,), dtype=torch.float32, device=dev)
    out = torch.empty((n, 3, H, W) if out_f32 else (n, H, W, 3), dtype=torch.float32 if out_f32 else torch.uint8,
                      device=dev)
    check(lib().nst_region_composite_u8(ys, hw, pr, len(sources), _arr(ctypes.c_int, nt), _arr(ctypes.c_int, ts),
                                        _arr(ctypes.c_float, tw), K, bx,
                                        orig_u8.data_ptr() if orig_u8 is not None else None, masks.data_ptr(), n, H,
                                        W, scratch.data_ptr() if scratch is not None else None, nfl,
                                        None if out_f32 else out.data_ptr(), out.data_ptr() if out_f32 else None,
                                        _stream(dev)), "nst_region_composite_u8")
    return out


def crop_input(frames_u8: torch.Tensor, box: Tuple[int, int, int, int], out_hw: Tuple[int, int]) -> torch.Tensor:
    """--region_optimize model input of one crop for a batch: [n,3,oh,ow] f32 in [0,1]."""
    n, H, W, _ = frames_u8.shape
    out = torch.empty((n, 3, out_hw[0], out_hw[1]), dtype=torch.float32, device=frames_u8.device)
    check(lib().nst_region_crop_input(frames_u8.data_ptr(), n, H, W, _arr(ctypes.c_int, box), out_hw[0], out_hw[1],
                                      out.data_ptr(), _stream(frames_u8.device)), "nst_region_crop_input")
    return out


def resized_source(y: torch.Tensor, preset: str, fit_hw: Tuple[int, int], out_hw: Tuple[int, int]) -> torch.Tensor:
    """The advanced path's low-resolution copy of a model output (pipeline.py:1786-1796): decoded, fitted to
    the content size, resized bilinearly -> decoded f32 [n,3,oh,ow] (a 'none'-preset source)."""
    n, _, h, w = y.shape
    out = torch.empty((n, 3, out_hw[0], out_hw[1]), dtype=torch.float32, device=y.device)
    check(lib().nst_region_resize(y.data_ptr(), n, h, w, _lib.PRESETS[preset], fit_hw[0], fit_hw[1], out_hw[0],
                                  out_hw[1], out.data_ptr(), _stream(y.device)), "nst_region_resize")
    return out


# ============================================================================ the pipeline's two region paths
def forward_raw(model, x: torch.Tensor, preset: str) -> torch.Tensor:
    """One nst_forward of a module-like model: x u8 NHWC frames or f32 NCHW [0,1] images -> raw f32 NCHW."""
    dev = x.device
    eng = model.engine(dev)
    if x.dtype == torch.uint8:
        n, h, w, _ = x.shape
        fmt = _lib.NST_IO_U8_NHWC
    else:
        n, _, h, w = x.shape
        fmt = _lib.NST_IO_F32_NCHW
    oh, ow = eng.output_hw(h, w)
    y = torch.empty((n, 3, oh, ow), dtype=torch.float32, device=dev)
    eng.forward_into(x.contiguous(), fmt, n, h, w, _lib.PRESETS[preset], y, _lib.NST_IO_F32_NCHW)
    return y


class RegionCompositor:
    """State of pipeline.py's region blending across the frames of one run (mask / config caches, parsed
    animations), for either path.  `args` is the pipeline's argparse namespace."""

    def __init__(self, args, device):
        self.a = args
        self.dev = torch.device(device)
        self.optimized = bool(getattr(args, "region_optimize", False))
        self.mode = args.region_mode
        self.feather = int(getattr(args, "region_feather", 20))
        self.rotate = float(getattr(args, "region_rotate", 0.0) or 0.0)
        morph_spec = getattr(args, "region_morph", None)
        self.morph = parse_morph_animation(morph_spec) if morph_spec else MorphAnimation(enabled=False)
        self.oc = float(getattr(args, "region_original", 0.0) or 0.0)
        self.blend_spec = getattr(args, "region_blend_spec", None)
        self.scale_spec = getattr(args, "region_scales", None)
        self.animating = self.rotate != 0 or self.morph.enabled
        self.seed = parse_region_seed(getattr(args, "region_seed", None), self.optimized, self.animating)
        self.cache: Dict[tuple, tuple] = {}
        self.blend_anims = None
        self.scale_anims = None
        self._anims_parsed = False

    # ---- masks: rotation + re-feather (region_blend.py:1757-1762) ----
    def _animate(self, masks, frame_idx):
        if self.rotate != 0:
            masks = feather_planes(rotate_planes(masks, frame_idx * self.rotate), self.feather // 2)
        if self.morph.enabled:  # region_blend.py:1765-1768
            masks = feather_planes(morph_planes(masks, self.morph, frame_idx), max(5, self.feather // 4))
        return masks

    # ---- standard path: every model styled the whole frame (pipeline.py:1720-1839) ----
    def standard(self, raw: List[Source], orig_u8: torch.Tensor, frame_ids: List[int], num_models_quirk: int,
                 fit_hw: Tuple[int, int], out_f32: bool = False) -> torch.Tensor:
        """raw[i]: output i of the compressed outputs list (A, then B..H in order) for the batch; frame_ids are
        the reference's 1-based frame indices.  -> u8 [n,H,W,3]."""
        a = self.a
        H, W = fit_hw
        n_out = len(raw)
        count = getattr(a, "region_count", None) or num_models_quirk
        assignment = getattr(a, "region_assignment", "random")
        animating = self.animating
        weights = None
        if assignment == "weighted":
            try:
                from .pipeline import parse_blend_weights
                weights = parse_blend_weights(getattr(a, "blend_models_weights", None), num_models_quirk)
            except Exception:
                weights = None
        advanced = bool(self.blend_spec or self.scale_spec)
        with_orig = self.oc > 0 or (advanced and bool(self.blend_spec) and "O" in self.blend_spec.upper())
        sources, scale_of = list(raw), {1.0: list(range(n_out))}
        if advanced:
            for s in get_required_scales(count, num_models_quirk, assignment, self.blend_spec, self.scale_spec,
                                         self.seed, self.oc):
                if s != 1.0:  # pipeline.py:1786-1796: the full outputs resized down, upsampled by the composite
                    hw = (int(H * s), int(W * s))
                    scale_of[s] = []
                    for r in raw:
                        sources.append(Source(resized_source(r.y, r.preset, (H, W), hw), "none"))
                        scale_of[s].append(len(sources) - 1)
            # dict order as the reference builds it (scale 1.0 entry is the first only if listed first)
        n_fr = orig_u8.shape[0]
        out = torch.empty((n_fr, 3, H, W) if out_f32 else (n_fr, H, W, 3),
                          dtype=torch.float32 if out_f32 else torch.uint8, device=self.dev)

        def configs_for(k_masks):
            if advanced:
                return parse_region_configs(k_masks, n_out, assignment, self.blend_spec, self.scale_spec, self.seed,
                                            self.oc)
            asg = assign_models_to_regions(k_masks, n_out, assignment, weights, self.seed, self.oc)
            return [RegionConfig([m], [1.0], 1.0) for m in asg]

        for j, fid in enumerate(frame_ids):
            if animating:  # cached masks + configs, rotated per frame (region_blend.py:1737-1762)
                key = (H, W, count, advanced)
                if key not in self.cache:
                    m = render_masks(draw_geometry(H, W, self.mode, count, self.seed), H, W, self.feather, self.dev)
                    self.cache[key] = (m, configs_for(m.shape[0]))
                base, cfgs = self.cache[key]
                masks = self._animate(base, fid)
            elif self.seed is not None:  # a fixed seed regenerates the same masks and configs every frame
                key = ("std", H, W, count, advanced)
                if key not in self.cache:
                    m = render_masks(draw_geometry(H, W, self.mode, count, self.seed), H, W, self.feather, self.dev)
                    self.cache[key] = (m, configs_for(m.shape[0]))
                masks, cfgs = self.cache[key]
            else:  # no seed: fresh random regions and assignments per frame
                masks = render_masks(draw_geometry(H, W, self.mode, count, self.seed), H, W, self.feather, self.dev)
                cfgs = configs_for(masks.shape[0])
            terms = []
            for c in cfgs:
                sc = c.scale
                if sc not in scale_of:
                    sc = min(list(scale_of.keys()), key=lambda s: abs(s - c.scale))
                tl = []
                for mi, w in zip(c.model_indices, c.model_weights):
                    if mi != -1 and not (0 <= mi < n_out):
                        raise NstError(f"region config names model {mi} but only {n_out} outputs exist")
                    if mi == -1 and not with_orig:
                        raise NstError("Region config uses original (-1) but no original frame provided")
                    tl.append((-1 if mi == -1 else scale_of[sc][mi], w))
                terms.append(tl)
            if fid <= 2 or fid % 50 == 0:
                print(f"[region] mode={self.mode} regions={masks.shape[0]} models={n_out} assignment={assignment} "
                      f"feather={self.feather}px seed={self.seed}", flush=True)
            if not animating and self.seed is not None:  # masks and terms shared by the batch: one launch
                return composite(sources, terms, masks, orig_u8 if with_orig else None, out_f32=out_f32)
            srcs_j = [Source(s.y[j:j + 1], s.preset) for s in sources]
            out[j:j + 1] = composite(srcs_j, terms, masks, orig_u8[j:j + 1] if with_orig else None, out_f32=out_f32)
        return out

    # ---- --region_optimize: crops styled per region (pipeline.py:1120-1407) ----
    def optimized_frames(self, slot_models: Dict[int, tuple], orig_u8: torch.Tensor, frame_ids: List[int],
                         out_f32: bool = False) -> torch.Tensor:
        """slot_models: letter index (A=0..H=7) -> (model, io_preset) of the loaded slots."""
        a = self.a
        n, H, W, _ = orig_u8.shape
        count = getattr(a, "region_count", None) or 4
        assignment = getattr(a, "region_assignment", "sequential")
        pad = int(getattr(a, "region_padding", 64))
        num_models = len(slot_models)
        sizes_spec = getattr(a, "region_sizes", None)
        key = ("opt", H, W, count)
        if key not in self.cache:
            sizes = parse_region_sizes(sizes_spec, count) if sizes_spec else None
            g = draw_geometry(H, W, self.mode, count, self.seed, sizes)
            masks = render_masks(g, H, W, self.feather, self.dev)
            cfgs = parse_region_configs(masks.shape[0], num_models, assignment, self.blend_spec, self.scale_spec,
                                        self.seed, self.oc)
            self.cache[key] = (masks, cfgs)
        base, cfgs = self.cache[key]
        with_orig = self.oc > 0 or bool(self.blend_spec and "O" in self.blend_spec.upper())
        if not self._anims_parsed:
            k = base.shape[0]
            bspec = getattr(a, "blend_animate_regions", None) or getattr(a, "blend_animate", None)
            sspec = getattr(a, "scale_animate_regions", None) or getattr(a, "scale_animate", None)
            self.blend_anims = parse_region_blend_animations(bspec, k) if bspec else None
            self.scale_anims = parse_region_scale_animations(sspec, k) if sspec else None
            self._anims_parsed = True
        out = torch.empty((n, 3, H, W) if out_f32 else (n, H, W, 3), dtype=torch.float32 if out_f32 else torch.uint8,
                          device=self.dev)
        # frames sharing masks, boxes and scales run as one batch per (region, model)
        plans, order = {}, []
        static_masks = None
        for j, fid in enumerate(frame_ids):
            if self.animating:
                masks = self._animate(base, fid)
                boxes = [(max(0, x1 - pad), max(0, y1 - pad), min(W, x2 + pad), min(H, y2 + pad))
                         for x1, y1, x2, y2 in mask_bboxes(masks)]
                mkey = ("rot", j)
            else:  # static masks: their padded boxes are computed once per run
                if static_masks is None:
                    bkey = ("opt-boxes", H, W, count, pad)
                    if bkey not in self.cache:
                        self.cache[bkey] = [(max(0, x1 - pad), max(0, y1 - pad), min(W, x2 + pad), min(H, y2 + pad))
                                            for x1, y1, x2, y2 in mask_bboxes(base)]
                    static_masks = (base, self.cache[bkey])
                masks, boxes = static_masks
                mkey = ("static",)
            scales = []
            for k, c in enumerate(cfgs):
                s = c.scale
                if self.scale_anims and k < len(self.scale_anims):
                    s = compute_animated_scale(s, fid, self.scale_anims[k])
                scales.append(s)
            wts = []
            for k, c in enumerate(cfgs):
                if self.blend_anims and k < len(self.blend_anims):
                    wts.append(compute_animated_weights(c.model_weights, fid, self.blend_anims[k]))
                else:
                    wts.append(c.model_weights)
            pk = (mkey, tuple(scales), tuple(tuple(w) for w in wts))
            if pk not in plans:
                plans[pk] = (masks, boxes, scales, wts, [])
                order.append(pk)
            plans[pk][4].append(j)
        for pk in order:
            masks, boxes, scales, wts, js = plans[pk]
            idx = torch.tensor(js, device=self.dev)
            frames = orig_u8 if len(js) == n else orig_u8.index_select(0, idx).contiguous()
            srcs, terms = [], []
            for k, c in enumerate(cfgs):
                x1, y1, x2, y2 = boxes[k]
                ch, cw = y2 - y1, x2 - x1
                s = scales[k]
                ih, iw = (max(1, int(ch * s)), max(1, int(cw * s))) if s < 1.0 else (ch, cw)
                tl = []
                crop = None
                for mi, w in zip(c.model_indices, wts[k]):
                    if mi == -1:
                        if not with_orig:
                            raise NstError("Region uses original but no original provided")
                        tl.append((-1, w))
                        continue
                    if mi not in slot_models:
                        raise NstError(f"Model {mi} not in styled_crops (model {chr(ord('A') + mi)} is not loaded)")
                    model, preset = slot_models[mi]
                    # pipeline.py:1363-1375: the crop path knows imagenet_255 and imagenet_01; every other preset
                    # runs as raw 0..255 in / y/255 out
                    preset = preset if preset in ("imagenet_255", "imagenet_01") else "raw_255"
                    if crop is None:
                        crop = crop_input(frames, (x1, y1, x2, y2), (ih, iw))
                    srcs.append(Source(forward_raw(model, crop, preset), preset))
                    tl.append((len(srcs) - 1, w))
                terms.append(tl)
            res = composite(srcs, terms, masks, frames if with_orig else None, boxes=boxes, out_f32=out_f32)
            if len(js) == n:
                out = res
            else:
                out.index_copy_(0, idx, res)
        return out
