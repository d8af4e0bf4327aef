"""Temporal stage of the frame loop on the MI355X engine: the flow-guided EMA
(--flow_ema, pipeline.py:1884-1940) and the motion-adaptive blend (--motion_blend, :2072-2086).

Per frame, in frame order (the EMA state is the previous fused frame):
  gray = pil_rgb.convert("L")                                   nst_gray_u8 (Pillow's integer luma)
  flow = cv2.calcOpticalFlowFarneback(prev_gray, gray, None, 0.5, 3, 15, 3, 5, 1.1, 0)   nst_flow_farneback
  out01 = clip(a * out01 + (1 - a) * warp(prev_styled01, flow))                         nst_flow_fuse
  prev_gray, prev_styled01 = gray, out01
and, when --motion_blend is on, the blend alpha from |flow| (nst_motion_alpha).

--flow_downscale ds computes the flow on INTER_AREA-reduced grays (an exact integer factor of the frame) and
brings it back with INTER_LINEAR x ds.  The reference's default --flow_method is DIS (cv2.DISOpticalFlow,
PRESET_FAST); only Farneback is built here, so a DIS request fails loudly (pipeline.reject_out_of_scope).  cv2 is not installed in this environment: the
Farneback, remap and GaussianBlur restatements are parity unpinned.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np
import torch

from . import _lib
from ._lib import check, lib

MOTION_NORM = 8.0  # pipeline.py:1075-1077
MIN_ALPHA = 0.40
GAUSS_SIGMA = 3.0
FARNEBACK = (0.5, 3, 15, 3, 5, 1.1)  # pipeline.py:1896-1899


def gray_u8(frames_u8: torch.Tensor) -> torch.Tensor:
    """[n,h,w,3] uint8 RGB -> [n,h,w] uint8 luma (Image.convert('L'))."""
    n, h, w, _ = frames_u8.shape
    out = torch.empty((n, h, w), dtype=torch.uint8, device=frames_u8.device)
    check(lib().nst_gray_u8(frames_u8.contiguous().data_ptr(), n, h, w, out.data_ptr(),
                            _lib.stream_ptr(frames_u8.device)), "nst_gray_u8")
    return out


class FlowScratch:
    def __init__(self):
        self.buf = None

    def get(self, h, w, device):
        sz = ctypes.c_size_t()
        check(lib().nst_flow_scratch_floats(h, w, ctypes.byref(sz)), "nst_flow_scratch_floats")
        if self.buf is None or self.buf.numel() < sz.value or self.buf.device != device:
            self.buf = torch.empty((sz.value,), dtype=torch.float32, device=device)
        return self.buf


def farneback(prev_gray: torch.Tensor, gray: torch.Tensor, scratch: Optional[FlowScratch] = None,
              params=FARNEBACK) -> torch.Tensor:
    """[h,w] uint8 x 2 -> flow [h,w,2] float32 (dx, dy)."""
    h, w = gray.shape
    dev = gray.device
    sc = (scratch or FlowScratch()).get(h, w, dev)
    flow = torch.empty((h, w, 2), dtype=torch.float32, device=dev)
    ps, lv, ws, it, pn, sg = params
    check(lib().nst_flow_farneback(prev_gray.contiguous().data_ptr(), gray.contiguous().data_ptr(), h, w, float(ps),
                                   int(lv), int(ws), int(it), int(pn), float(sg), flow.data_ptr(), sc.data_ptr(),
                                   sc.numel(), _lib.stream_ptr(dev)), "nst_flow_farneback")
    return flow


def fuse(curr01: torch.Tensor, prev01: torch.Tensor, flow: torch.Tensor, alpha: float) -> torch.Tensor:
    """[3,h,w] float32 planes -> clip(a*curr + (1-a)*warp(prev, flow))."""
    _, h, w = curr01.shape
    a = float(max(0.0, min(1.0, alpha)))
    out = torch.empty_like(curr01)
    check(lib().nst_flow_fuse(curr01.contiguous().data_ptr(), prev01.contiguous().data_ptr(), flow.data_ptr(), h, w,
                              float(np.float32(a)), float(np.float32(1.0 - a)), out.data_ptr(),
                              _lib.stream_ptr(curr01.device)), "nst_flow_fuse")
    return out


def motion_alpha(flow: torch.Tensor, blend: float) -> torch.Tensor:
    """pipeline.py:2073-2080: [h,w] float32 alpha = blend - (blend - 0.4) * GaussianBlur(clip(|flow|/8), 3)."""
    h, w, _ = flow.shape
    alpha = torch.empty((h, w), dtype=torch.float32, device=flow.device)
    tmp = torch.empty_like(alpha)
    check(lib().nst_motion_alpha(flow.data_ptr(), h, w, float(MOTION_NORM), float(GAUSS_SIGMA), float(np.float32(blend)),
                                 float(np.float32(float(blend) - MIN_ALPHA)), alpha.data_ptr(), tmp.data_ptr(),
                                 _lib.stream_ptr(flow.device)), "nst_motion_alpha")
    return alpha


def downscale_gray(gray: torch.Tensor, ds: int) -> torch.Tensor:
    """cv2.resize(gray, (W // ds, H // ds), interpolation=cv2.INTER_AREA) at an exact integer factor."""
    h, w = gray.shape
    out = torch.empty((h // ds, w // ds), dtype=torch.uint8, device=gray.device)
    check(lib().nst_flow_downscale_gray(gray.contiguous().data_ptr(), h, w, int(ds), out.data_ptr(),
                                        _lib.stream_ptr(gray.device)), "nst_flow_downscale_gray")
    return out


def upscale_flow(flow_small: torch.Tensor, h: int, w: int, ds: int) -> torch.Tensor:
    """cv2.resize(flow_small, (W, H), INTER_LINEAR) * ds (pipeline.py:1920-1922)."""
    hs, ws, _ = flow_small.shape
    out = torch.empty((h, w, 2), dtype=torch.float32, device=flow_small.device)
    check(lib().nst_flow_upscale(flow_small.contiguous().data_ptr(), hs, ws, h, w, float(ds), out.data_ptr(),
                                 _lib.stream_ptr(flow_small.device)), "nst_flow_upscale")
    return out


def planar_to_u8(out01: torch.Tensor) -> torch.Tensor:
    """ToPILImage of float planes [n,3,h,w] in [0,1]: pic.mul(255).byte() -> [n,h,w,3] uint8."""
    n, _, h, w = out01.shape
    out = torch.empty((n, h, w, 3), dtype=torch.uint8, device=out01.device)
    check(lib().nst_decode_resize_u8(out01.contiguous().data_ptr(), n, h, w, _lib.PRESETS["none"], out.data_ptr(), h, w,
                                     _lib.stream_ptr(out01.device)), "nst_decode_resize_u8")
    return out


class FlowSmoother:
    """The reference's temporal caches (prev_gray, prev_styled01, last_flow; reset on a frame-size change)."""

    def __init__(self, flow_ema: bool, flow_alpha: float, downscale: int = 1):
        self.enabled = flow_ema
        self.alpha = flow_alpha
        self.ds = max(1, int(downscale))
        self.scratch = FlowScratch()
        self.reset()

    def reset(self):
        self.prev_gray = None
        self.prev_styled = None
        self.last_flow = None

    def __call__(self, out01: torch.Tensor, orig_u8: torch.Tensor) -> torch.Tensor:
        """One frame: out01 [3,h,w] float32 (pre-LAB styled frame), orig_u8 [h,w,3] -> fused out01."""
        gray = gray_u8(orig_u8[None])[0]
        self.last_flow = None
        if self.enabled and self.prev_gray is not None and self.prev_styled is not None:
            if self.prev_gray.shape == gray.shape:
                if self.ds > 1:  # pipeline.py:1886-1892, 1920-1923
                    h, w = gray.shape
                    small = farneback(downscale_gray(self.prev_gray, self.ds), downscale_gray(gray, self.ds), self.scratch)
                    flow = upscale_flow(small, h, w, self.ds)
                else:
                    flow = farneback(self.prev_gray, gray, self.scratch)
                out01 = fuse(out01, self.prev_styled, flow, self.alpha)
                self.last_flow = flow
        self.prev_gray = gray
        self.prev_styled = out01
        return out01
