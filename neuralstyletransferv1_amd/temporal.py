"""Temporal stage of the frame loop on the MI355X engine: the flow-guided EMA
(--flow_ema, pipeline.py:1884-1940) and the motion-adaptive blend (--motion_blend, :2072-2086).

Per frame, in frame order (the EMA state is the previous fused frame):
  gray = pil_rgb.convert("L")                                   nst_gray_u8 (Pillow's integer luma)
  flow = cv2.DISOpticalFlow_create(PRESET_FAST).calc(prev_gray, gray, None)      nst_flow_dis (default, :1904-1914)
       | cv2.calcOpticalFlowFarneback(prev_gray, gray, None, 0.5, 3, 15, 3, 5, 1.1, 0)   nst_flow_farneback
  out01 = clip(a * out01 + (1 - a) * warp(prev_styled01, flow))                         nst_flow_fuse
  prev_gray, prev_styled01 = gray, out01
and, when --motion_blend is on, the blend alpha from |flow| (nst_motion_alpha).  The flows depend only on the
original frames, so a batch's flows are computed together (DIS: one call for all its frame pairs) before the
sequential fuse.

--flow_downscale ds computes the flow on INTER_AREA-reduced grays of (W // ds, H // ds) (any factor: cv2's
fractional area cells when ds does not divide the frame) and brings it back with INTER_LINEAR x ds.  cv2 is not
installed in this environment: the DIS, Farneback, INTER_AREA, remap and GaussianBlur restatements are parity
unpinned.
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


class DisScratch:
    def __init__(self):
        self.buf = None

    def get(self, n, h, w, device):
        sz = ctypes.c_size_t()
        check(lib().nst_flow_dis_scratch_bytes(n, h, w, ctypes.byref(sz)), "nst_flow_dis_scratch_bytes")
        if self.buf is None or self.buf.numel() < sz.value or self.buf.device != device:
            self.buf = torch.empty((max(sz.value, 256),), dtype=torch.uint8, device=device)
        return self.buf


def dis_supported(h: int, w: int) -> bool:
    """Whether nst_flow_dis accepts h x w grays (the frame-size limits of dis_check_shape: a coarsest pyramid
    level at or above the finest, a stripe buffer that fits LDS); host-side, no GPU work."""
    if h <= 0 or w <= 0:
        return False
    sz = ctypes.c_size_t()
    return lib().nst_flow_dis_scratch_bytes(1, h, w, ctypes.byref(sz)) == _lib.NST_OK


def dis(prev_gray: torch.Tensor, gray: torch.Tensor, scratch: Optional[DisScratch] = None) -> torch.Tensor:
    """cv2.DISOpticalFlow_create(PRESET_FAST).calc of frame pairs: [n,h,w] (or [h,w]) uint8 x 2 -> flow
    [n,h,w,2] (or [h,w,2]) float32 (dx, dy)."""
    single = gray.dim() == 2
    p = prev_gray[None] if single else prev_gray
    g = gray[None] if single else gray
    n, h, w = g.shape
    dev = g.device
    sc = (scratch or DisScratch()).get(n, h, w, dev)
    flow = torch.empty((n, h, w, 2), dtype=torch.float32, device=dev)
    check(lib().nst_flow_dis(p.contiguous().data_ptr(), g.contiguous().data_ptr(), n, h, w, flow.data_ptr(),
                             sc.data_ptr(), sc.numel(), _lib.stream_ptr(dev)), "nst_flow_dis")
    return flow[0] if single else flow


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
    """cv2.resize(gray, (W // ds, H // ds), interpolation=cv2.INTER_AREA) (pipeline.py:1886-1889: floored sizes,
    any factor)."""
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

    def __init__(self, flow_ema: bool, flow_alpha: float, downscale: int = 1, method: str = "dis"):
        if method not in ("dis", "farneback"):
            raise _lib.NstError(f"flow method must be dis or farneback, got {method!r}")
        self.enabled = flow_ema
        self.alpha = flow_alpha
        self.ds = max(1, int(downscale))
        self.method = method
        self.scratch = FlowScratch()
        self.dis_scratch = DisScratch()
        self._warned = False
        self.reset()

    def flows(self, prev_gray: torch.Tensor, grays: torch.Tensor) -> Optional[torch.Tensor]:
        """Flows of the pairs (prev, grays[0]), (grays[0], grays[1]), ... -> [n,h,w,2] (pipeline.py:1886-1923:
        optional INTER_AREA reduction by ds, the flow, INTER_LINEAR back x ds), or None when DIS cannot run on
        the (reduced) frame size: the reference wraps dis.calc in try/except and skips the flow for that frame
        (pipeline.py:1903-1917), so the frames pass through unfused."""
        prevs = torch.cat([prev_gray[None], grays[:-1]], dim=0)
        n, h, w = grays.shape
        if self.method == "dis" and not dis_supported(h // self.ds, w // self.ds):
            if not self._warned:
                print(f"[flow][warn] DIS cannot run on {w // self.ds}x{h // self.ds} frames; skipping the flow")
                self._warned = True
            return None
        if self.ds > 1:
            prevs = torch.stack([downscale_gray(g, self.ds) for g in prevs])
            cur = torch.stack([downscale_gray(g, self.ds) for g in grays])
        else:
            cur = grays
        if self.method == "dis":
            small = dis(prevs, cur, self.dis_scratch)
        else:
            small = torch.stack([farneback(prevs[k], cur[k], self.scratch) for k in range(n)])
        if self.ds > 1:
            return torch.stack([upscale_flow(small[k], h, w, self.ds) for k in range(n)])
        return small

    def batch(self, out01: torch.Tensor, orig_u8: torch.Tensor):
        """A batch of frames in order: out01 [n,3,h,w], orig_u8 [n,h,w,3] -> (fused out01 list, flow list; None
        where a frame has no predecessor of its size)."""
        n, _, h, w = out01.shape
        grays = gray_u8(orig_u8)
        fl = None
        if self.enabled and self.prev_gray is not None and self.prev_gray.shape == grays.shape[1:]:
            fl = self.flows(self.prev_gray, grays)
        elif self.enabled and n > 1:
            fl = self.flows(grays[0], grays[1:])
            fl = None if fl is None else [None] + list(fl)
        fused, flows = [], []
        for k in range(n):
            f = None if fl is None else fl[k]
            o = out01[k]
            if f is not None and self.prev_styled is not None and self.prev_styled.shape == o.shape:
                o = fuse(o, self.prev_styled, f, self.alpha)
            else:
                f = None
            fused.append(o)
            flows.append(f)
            self.prev_styled = o
        self.prev_gray = grays[-1]
        self.last_flow = flows[-1]
        return fused, flows

    def reset(self):
        self.prev_gray = None
        self.prev_styled = None
        self.last_flow = None

    def __call__(self, out01: torch.Tensor, orig_u8: torch.Tensor) -> torch.Tensor:
        """One frame: out01 [3,h,w] float32 (pre-LAB styled frame), orig_u8 [h,w,3] -> fused out01."""
        gray = gray_u8(orig_u8[None])[0]
        self.last_flow = None
        if self.enabled and self.prev_gray is not None and self.prev_styled is not None:
            fl = self.flows(self.prev_gray, gray[None]) if self.prev_gray.shape == gray.shape else None
            if fl is not None:
                out01 = fuse(out01, self.prev_styled, fl[0], self.alpha)
                self.last_flow = fl[0]
        self.prev_gray = gray
        self.prev_styled = out01
        return out01
