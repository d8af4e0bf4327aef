"""GPU post chain of the per-frame loop (pipeline.py:1942-2092) over libnst_hip kernels.

* `LabSmoother`: LAB lightness/chroma EMA (pipeline.py:1942-1978).  Pillow routes RGB<->LAB
  through LittleCMS (8-bit LAB: L 0..255, a/b signed bytes stored as uint8); both transforms
  are per-pixel, so each is exactly one 2^24-entry table.  The tables are made ONCE from
  Pillow itself (the reference's own dependency) and gathered on the GPU per pixel; the EMA
  state (prev_L, prev_a, prev_b) lives in HBM as fp32.
* `blend_frames`: mask composite (pipeline.py:2040-2043) + uniform blend (:2087-2092) + the
  final ToPILImage truncation.
"""
from __future__ import annotations

import ctypes
import threading
from typing import Optional

import numpy as np
import torch

from . import _lib
from ._lib import check, lib

_LUT_LOCK = threading.Lock()
_LUTS: Optional[tuple] = None


def pillow_lab_luts() -> tuple:
    """(rgb2lab, lab2rgb) as uint8 [2^24*3] numpy arrays, built from Pillow/LittleCMS."""
    global _LUTS
    with _LUT_LOCK:
        if _LUTS is None:
            from PIL import Image
            idx = np.arange(1 << 24, dtype=np.uint32)
            grid = np.stack([(idx >> 16) & 255, (idx >> 8) & 255, idx & 255], -1).astype(np.uint8)
            grid = grid.reshape(4096, 4096, 3)
            rgb2lab = np.ascontiguousarray(np.array(Image.fromarray(grid, "RGB").convert("LAB")).reshape(-1))
            lab2rgb = np.ascontiguousarray(
                np.array(Image.frombytes("LAB", (4096, 4096), grid.tobytes()).convert("RGB")).reshape(-1))
            _LUTS = (rgb2lab, lab2rgb)
        return _LUTS


class LabTables:
    """Device copy of the two LittleCMS tables (nst_lab handle)."""

    def __init__(self, device: torch.device):
        rgb2lab, lab2rgb = pillow_lab_luts()
        h = ctypes.c_void_p()
        idx = device.index if device.index is not None else torch.cuda.current_device()
        check(lib().nst_lab_create(rgb2lab.ctypes.data, lab2rgb.ctypes.data, idx, ctypes.byref(h)), "nst_lab_create")
        self._h = h
        self.device = device

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().nst_lab_destroy(h)
            except Exception:
                pass


_TABLES = {}


def lab_tables(device: torch.device) -> LabTables:
    key = (device.type, device.index)
    if key not in _TABLES:
        _TABLES[key] = LabTables(device)
    return _TABLES[key]


class LabSmoother:
    """Stateful LAB EMA over a frame sequence (frames in order, possibly in batches)."""

    def __init__(self, device, smooth_lightness=True, smooth_alpha=0.7, smooth_chroma=False, chroma_alpha=0.85):
        self.device = torch.device(device)
        self.sl, self.sc = bool(smooth_lightness), bool(smooth_chroma)
        # numpy: python-float * float32 array computes in float32 with the scalar cast to float32
        self.a, self.oma = np.float32(smooth_alpha), np.float32(1.0 - smooth_alpha)
        self.ca, self.coma = np.float32(chroma_alpha), np.float32(1.0 - chroma_alpha)
        self.state: Optional[torch.Tensor] = None
        self.hw = None

    def reset(self):
        self.state = None
        self.hw = None

    def __call__(self, frames_u8: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        _lib.require_gpu_tensor(frames_u8, "frames")
        if not (self.sl or self.sc):
            return frames_u8
        frames_u8 = frames_u8.contiguous()
        n, h, w, _ = frames_u8.shape
        first = 0
        if self.state is None or self.hw != (h, w):  # pipeline.py:1104-1113 resets caches on size change
            self.state = torch.zeros(3 * h * w, dtype=torch.float32, device=self.device)
            self.hw = (h, w)
            first = 1
        if out is None:
            out = torch.empty_like(frames_u8)
        t = lab_tables(self.device)
        check(lib().nst_lab_ema_u8(t._h, frames_u8.data_ptr(), out.data_ptr(), n, h, w, int(self.sl), float(self.a),
                                   float(self.oma), int(self.sc), float(self.ca), float(self.coma),
                                   self.state.data_ptr(), first, _lib.stream_ptr(self.device)), "nst_lab_ema_u8")
        return out

    # ---- the same EMA in three stages for the sharded pipeline (nst_lab_planes_u8 / _ema_planes / _merge_u8):
    # the owner of a frame extracts the planes the EMA reads, the ordered stage smooths them in frame order, the
    # owner puts them back; bytes identical to __call__ on the same frames in the same order
    @property
    def nplanes(self) -> int:
        return int(self.sl) + 2 * int(self.sc)

    def planes(self, frames_u8: torch.Tensor) -> torch.Tensor:
        """[n,h,w,3] uint8 -> [n, nplanes, h*w] uint8 LAB planes (L, then a, b) of the smoothed channels."""
        _lib.require_gpu_tensor(frames_u8, "frames")
        frames_u8 = frames_u8.contiguous()
        n, h, w, _ = frames_u8.shape
        out = torch.empty((n, self.nplanes, h * w), dtype=torch.uint8, device=frames_u8.device)
        if n:
            t = lab_tables(frames_u8.device)
            check(lib().nst_lab_planes_u8(t._h, frames_u8.data_ptr(), n, h, w, int(self.sl), int(self.sc),
                                          out.data_ptr(), _lib.stream_ptr(frames_u8.device)), "nst_lab_planes_u8")
        return out

    def smooth_planes(self, planes: torch.Tensor, hw: tuple) -> torch.Tensor:
        """The ordered stage: [n, nplanes, h*w] planes of consecutive frames of size hw -> smoothed planes (state
        carried across calls, reset on a size change like __call__)."""
        _lib.require_gpu_tensor(planes, "planes")
        planes = planes.contiguous()
        n = planes.shape[0]
        h, w = hw
        first = 0
        if self.state is None or self.hw != (h, w):
            self.state = torch.zeros(3 * h * w, dtype=torch.float32, device=self.device)
            self.hw = (h, w)
            first = 1
        out = torch.empty_like(planes)
        check(lib().nst_lab_ema_planes(planes.data_ptr(), out.data_ptr(), n, h, w, int(self.sl), float(self.a),
                                       float(self.oma), int(self.sc), float(self.ca), float(self.coma),
                                       self.state.data_ptr(), first, _lib.stream_ptr(self.device)),
              "nst_lab_ema_planes")
        return out

    def merge(self, frames_u8: torch.Tensor, planes: torch.Tensor) -> torch.Tensor:
        """The owner's last stage: frames with their smoothed planes put back (LAB -> RGB)."""
        _lib.require_gpu_tensor(frames_u8, "frames")
        frames_u8, planes = frames_u8.contiguous(), planes.to(frames_u8.device).contiguous()
        n, h, w, _ = frames_u8.shape
        if planes.shape != (n, self.nplanes, h * w):
            raise _lib.NstError(f"planes {tuple(planes.shape)} do not match frames {tuple(frames_u8.shape)}")
        out = torch.empty_like(frames_u8)
        if n:
            t = lab_tables(frames_u8.device)
            check(lib().nst_lab_merge_u8(t._h, frames_u8.data_ptr(), planes.data_ptr(), n, h, w, int(self.sl),
                                         int(self.sc), out.data_ptr(), _lib.stream_ptr(frames_u8.device)),
                  "nst_lab_merge_u8")
        return out


def blend_frames(styled_u8: torch.Tensor, orig_u8: torch.Tensor, blend: float = 1.0,
                 mask: Optional[torch.Tensor] = None, composite_mode: str = "keep") -> torch.Tensor:
    """[n,h,w,3] uint8 styled/original (+ optional [n,h,w] fp32 alpha, or uint8 mask read as m / 255)
    -> [n,h,w,3] uint8."""
    _lib.require_gpu_tensor(styled_u8, "styled")
    _lib.require_gpu_tensor(orig_u8, "orig")
    if styled_u8.shape != orig_u8.shape:
        raise _lib.NstError(f"styled {tuple(styled_u8.shape)} and original {tuple(orig_u8.shape)} differ")
    styled_u8, orig_u8 = styled_u8.contiguous(), orig_u8.contiguous()
    n, h, w, _ = styled_u8.shape
    mptr = None
    out = torch.empty_like(styled_u8)
    mode = 0 if composite_mode == "keep" else 1
    if mask is not None and mask.dtype == torch.uint8:  # 8-bit mask (DeepLab / PNG bytes): alpha = m / 255 fused
        _lib.require_gpu_tensor(mask, "mask")
        mask = mask.contiguous()
        if mask.numel() != n * h * w:
            raise _lib.NstError("mask must be [n,h,w]")
        check(lib().nst_blend_mask8_u8(styled_u8.data_ptr(), orig_u8.data_ptr(), mask.data_ptr(), mode,
                                       float(np.float32(blend)), float(np.float32(1.0 - blend)), out.data_ptr(), n, h, w,
                                       _lib.stream_ptr(styled_u8.device)), "nst_blend_mask8_u8")
        return out
    if mask is not None:
        mask = mask.to(styled_u8.device, torch.float32).contiguous()
        if mask.numel() != n * h * w:
            raise _lib.NstError("mask must be [n,h,w] alpha")
        mptr = mask.data_ptr()
    check(lib().nst_blend_u8(styled_u8.data_ptr(), orig_u8.data_ptr(), mptr, mode, float(np.float32(blend)),
                             float(np.float32(1.0 - blend)), out.data_ptr(), n, h, w,
                             _lib.stream_ptr(styled_u8.device)), "nst_blend_u8")
    return out


def blend_models_lab(frames_u8, weights_rest, w_l: float = 0.5, w_ab: float = 0.5) -> torch.Tensor:
    """LAB multi-model blend (pipeline.py:1841-1870) of [n,h,w,3] uint8 model outputs (A first).

    L comes from A; a/b = clip(wL*a_A + wab*sum_i w_i*a_i, 0, 255) on the raw LAB bytes, truncated.
    `weights_rest` pairs with frames_u8[1:] in zip order (the reference's zip(outputs[1:], ...))."""
    frames = [f.contiguous() for f in frames_u8]
    for f in frames:
        _lib.require_gpu_tensor(f, "frames")
        if f.shape != frames[0].shape or f.dtype != torch.uint8:
            raise _lib.NstError(f"LAB blend needs equal uint8 frames, got {tuple(f.shape)} vs {tuple(frames[0].shape)}")
    n, h, w, _ = frames[0].shape
    out = torch.empty_like(frames[0])
    m = len(frames)
    fp = (ctypes.c_void_p * m)(*[f.data_ptr() for f in frames])
    wr = [float(np.float32(x)) for x in weights_rest]
    wp = (ctypes.c_float * max(1, len(wr)))(*wr)
    t = lab_tables(frames[0].device)
    check(lib().nst_blend_models_lab_u8(t._h, fp, m, wp, len(wr), float(np.float32(w_l)), float(np.float32(w_ab)),
                                        n, h, w, out.data_ptr(), _lib.stream_ptr(frames[0].device)),
          "nst_blend_models_lab_u8")
    return out


def feather_masks(masks_u8: torch.Tensor, feather_px: int) -> torch.Tensor:
    """[n,h,w] uint8 fitted masks -> [n,h,w] fp32 alpha with the reference's Gaussian feather
    (pipeline.py:349-353: sigma = feather_px * 0.5; feather_px <= 0 -> plain m / 255)."""
    _lib.require_gpu_tensor(masks_u8, "masks")
    masks_u8 = masks_u8.contiguous()
    n, h, w = masks_u8.shape
    alpha = torch.empty((n, h, w), dtype=torch.float32, device=masks_u8.device)
    if not feather_px or feather_px <= 0:
        raise _lib.NstError("feather_masks needs feather_px > 0 (unfeathered masks are m / 255 on the host)")
    scratch = torch.empty_like(alpha)
    check(lib().nst_mask_feather(masks_u8.data_ptr(), n, h, w, float(feather_px) * 0.5, scratch.data_ptr(),
                                 alpha.data_ptr(), _lib.stream_ptr(masks_u8.device)), "nst_mask_feather")
    return alpha
