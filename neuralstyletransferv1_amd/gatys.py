"""Gatys neural style transfer by image optimisation (BASELINE.json configs[2]) on libnst_hip.

The reference has only the helpers this loop is built from -- `gram_matrix` (utils.py:80-83) and
`preprocess_for_vgg` (utils.py:93-96) -- and no VGG network, loss or optimiser.
This module provides the loop the configuration names, on hand-written HIP kernels through the
C ABI (include/nst_hip.h, nst_vgg_* / nst_gatys_* / nst_adam_step):

  * `VGG19Features`: the torchvision `vgg19().features` module layout (state_dict keys
    features.N.weight/bias), parameters as containers; `features(image)` runs the forward;
  * `Gatys`: content/style targets, loss + gradient with respect to the image, Adam;
  * `run_style_transfer(...)`: the usual loop (content-initialised image, `steps` Adam updates).

Loss (Gatys et al.): style = sum_l w_l * mean((G_l - A_l)^2) over relu1_1..relu5_1 with G = the
reference's gram_matrix of the ReLU feature map; content = mean((F - P)^2) at relu4_2; total =
content_weight * content + style_weight * style.  bf16 activations, fp32 accumulation.
Parity: against a torch-CPU fp32 restatement (oracle/gatys_oracle.py) -- unpinned by the
reference, which has no such loop.
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
from torch import nn

from . import _lib
from ._lib import NstError, NstParam, check, lib

STYLE_LAYERS = ("relu1_1", "relu2_1", "relu3_1", "relu4_1", "relu5_1")
CONTENT_LAYER = "relu4_2"
_CONV_IDX = (0, 2, 5, 7, 10, 12, 14, 16, 19, 21, 23, 25, 28)


class VGG19Features(nn.Module):
    """torchvision vgg19().features up to conv5_1 (the layers the loss needs); state_dict keys
    features.N.weight / features.N.bias as in torchvision's full model."""

    def __init__(self):
        super().__init__()
        cfg = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512]
        layers: List[nn.Module] = []
        cin = 3
        for v in cfg:
            if v == "M":
                layers.append(nn.MaxPool2d(2, 2))
            else:
                layers += [nn.Conv2d(cin, v, 3, padding=1), nn.ReLU(inplace=True)]
                cin = v
        self.features = nn.Sequential(*layers)

    def forward(self, x):  # noqa: D401 -- containers only
        raise NstError("VGG19Features runs through Gatys / libnst_hip (no torch forward)")


class Gatys:
    """One VGG-19 handle on one device plus the buffers of an h x w optimisation."""

    def __init__(self, state: Dict[str, torch.Tensor], device: torch.device, generic_only: bool = False):
        """generic_only: every conv on the generic implicit-GEMM kernel (NST_VGG_GENERIC_ONLY) instead of
        conv2_1 onward on the K-streaming GEMM conv; the same arithmetic summed in another order."""
        device = torch.device(device)
        if device.type != "cuda":
            raise NstError("the Gatys loop runs on MI355X (cuda) devices only; there is no CPU path")
        self.device = device
        host = {k: v.detach().to("cpu", torch.float32).contiguous() for k, v in state.items()}
        arr = (NstParam * len(host))()
        keep = []
        for i, (k, v) in enumerate(host.items()):
            b = k.encode()
            keep.append(b)
            arr[i].name = b
            arr[i].data = ctypes.cast(v.data_ptr(), ctypes.POINTER(ctypes.c_float))
            arr[i].numel = v.numel()
        h = ctypes.c_void_p()
        idx = device.index if device.index is not None else torch.cuda.current_device()
        flags = _lib.NST_VGG_GENERIC_ONLY if generic_only else 0
        check(lib().nst_vgg_create_ex(arr, len(host), idx, flags, ctypes.byref(h)), "nst_vgg_create")
        self._h = h
        self._hw: Optional[Tuple[int, int]] = None       # size of the scratch workspace
        self._tgt_hw: Optional[Tuple[int, int]] = None   # size the content / style targets were made for

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().nst_vgg_destroy(h)
            except Exception:
                pass

    def _sizes(self, hgt: int, wid: int) -> Tuple[int, int]:
        ws, stt = ctypes.c_size_t(), ctypes.c_size_t()
        check(lib().nst_gatys_buffer_bytes(self._h, hgt, wid, ctypes.byref(ws), ctypes.byref(stt)),
              "nst_gatys_buffer_bytes")
        return ws.value, stt.value

    def _workspace(self, hgt: int, wid: int) -> torch.Tensor:
        """Scratch for an h x w pass; the targets (self.state) are kept apart, so a features() call at another
        size does not invalidate them."""
        if self._hw != (hgt, wid):
            self.ws = torch.empty(self._sizes(hgt, wid)[0], dtype=torch.uint8, device=self.device)
            self.losses = torch.zeros(4, dtype=torch.float32, device=self.device)
            self._hw = (hgt, wid)
        self.ws.record_stream(torch.cuda.current_stream(self.device))
        return self.ws

    def _targets(self, hgt: int, wid: int) -> torch.Tensor:
        if self._tgt_hw != (hgt, wid):
            raise NstError(f"call set_targets for {hgt}x{wid} first (targets are for {self._tgt_hw})")
        return self.state

    @staticmethod
    def _image(x: torch.Tensor) -> torch.Tensor:
        _lib.require_gpu_tensor(x, "image")
        if x.dim() != 4 or x.shape[0] != 1 or x.shape[1] != 3:
            raise NstError(f"expected a [1,3,H,W] image, got {tuple(x.shape)}")
        return x.to(torch.float32).contiguous()

    def features(self, image: torch.Tensor) -> Dict[str, torch.Tensor]:
        """Rectified feature maps relu1_1 .. relu5_1, relu4_2 (bf16, NCHW view of the NHWC buffers)."""
        image = self._image(image)
        _, _, hgt, wid = image.shape
        ws = self._workspace(hgt, wid)
        shapes = [(hgt, wid, 64), (hgt // 2, wid // 2, 128), (hgt // 4, wid // 4, 256), (hgt // 8, wid // 8, 512),
                  (hgt // 16, wid // 16, 512), (hgt // 8, wid // 8, 512)]
        outs = [torch.empty(s, dtype=torch.bfloat16, device=self.device) for s in shapes]
        ptrs = (ctypes.c_void_p * 6)(*[o.data_ptr() for o in outs])
        check(lib().nst_vgg_features(self._h, image.data_ptr(), hgt, wid, ptrs, ws.data_ptr(), ws.numel(),
                                     _lib.stream_ptr(self.device)), "nst_vgg_features")
        names = STYLE_LAYERS + (CONTENT_LAYER,)
        return {n: o.permute(2, 0, 1).unsqueeze(0) for n, o in zip(names, outs)}

    def set_targets(self, content: torch.Tensor, style: torch.Tensor) -> None:
        content, style = self._image(content), self._image(style)
        if content.shape != style.shape:
            raise NstError("resize the style image to the content size first (same h x w)")
        _, _, hgt, wid = content.shape
        ws = self._workspace(hgt, wid)
        if self._tgt_hw != (hgt, wid):
            self.state = torch.empty(self._sizes(hgt, wid)[1], dtype=torch.uint8, device=self.device)
        stt = self.state
        self._tgt_hw = (hgt, wid)
        check(lib().nst_gatys_targets(self._h, content.data_ptr(), style.data_ptr(), hgt, wid, stt.data_ptr(),
                                      ws.data_ptr(), ws.numel(), _lib.stream_ptr(self.device)), "nst_gatys_targets")

    def grad(self, image: torch.Tensor, content_weight: float = 1.0, style_weight: float = 1e6,
             style_layer_weights: Sequence[float] = (1.0,) * 5) -> Tuple[torch.Tensor, torch.Tensor]:
        """-> (dL/d normalised image [1,3,h,w] fp32, losses [total, content, style] fp32 on device)."""
        image = self._image(image)
        g = torch.empty_like(image)
        self._grad_into(image, g, self.losses_for(image), content_weight, style_weight, style_layer_weights)
        return g, self.losses[:3].clone()

    def losses_for(self, image: torch.Tensor) -> torch.Tensor:
        self._workspace(image.shape[2], image.shape[3])
        return self.losses

    def _grad_into(self, image: torch.Tensor, g: torch.Tensor, losses: torch.Tensor, content_weight: float,
                   style_weight: float, style_layer_weights: Sequence[float]) -> None:
        """nst_gatys_grad into caller-owned buffers: g ([1,3,h,w] fp32) and losses (3 contiguous fp32 on the
        device), so the optimisation loop writes each step's losses straight into its trajectory row."""
        _, _, hgt, wid = image.shape
        stt = self._targets(hgt, wid)
        ws = self._workspace(hgt, wid)
        if losses.dtype != torch.float32 or losses.numel() < 3 or not losses.is_contiguous():
            raise NstError("losses: 3 contiguous fp32 values")
        wl = (ctypes.c_float * 5)(*[float(v) for v in style_layer_weights])
        check(lib().nst_gatys_grad(self._h, image.data_ptr(), hgt, wid, wl, float(content_weight), float(style_weight),
                                   stt.data_ptr(), g.data_ptr(), losses.data_ptr(), ws.data_ptr(), ws.numel(),
                                   _lib.stream_ptr(self.device)), "nst_gatys_grad")

    def grad_capture(self, image: torch.Tensor, content_weight: float = 1.0, style_weight: float = 1e6,
                     style_layer_weights: Sequence[float] = (1.0,) * 5):
        """grad() plus dL/dz of each of the 13 convs (z = pre-activation), bf16 [1,c,h,w] views."""
        image = self._image(image)
        _, _, hgt, wid = image.shape
        stt = self._targets(hgt, wid)
        ws = self._workspace(hgt, wid)
        shapes, hh, ww = [], hgt, wid
        for k, c in enumerate((64, 64, 128, 128, 256, 256, 256, 256, 512, 512, 512, 512, 512)):
            shapes.append((hh, ww, c))
            if k in (1, 3, 7, 11):
                hh, ww = hh // 2, ww // 2
        dz = [torch.zeros(s, dtype=torch.bfloat16, device=self.device) for s in shapes]
        ptrs = (ctypes.c_void_p * 13)(*[t.data_ptr() for t in dz])
        g = torch.empty_like(image)
        wl = (ctypes.c_float * 5)(*[float(v) for v in style_layer_weights])
        check(lib().nst_gatys_grad_capture(self._h, image.data_ptr(), hgt, wid, wl, float(content_weight),
                                           float(style_weight), stt.data_ptr(), g.data_ptr(), self.losses.data_ptr(),
                                           ws.data_ptr(), ws.numel(), ptrs, _lib.stream_ptr(self.device)),
              "nst_gatys_grad_capture")
        return g, self.losses[:3].clone(), [t.permute(2, 0, 1).unsqueeze(0) for t in dz]

    def adam(self, image: torch.Tensor, grad: torch.Tensor, m: torch.Tensor, v: torch.Tensor, step: int,
             lr: float, betas=(0.9, 0.999), eps: float = 1e-8, clamp01: bool = True) -> None:
        """In-place Adam update of `image` from nst_gatys_grad's gradient (torch.optim.Adam rule)."""
        _, c, hgt, wid = image.shape
        check(lib().nst_adam_step(image.data_ptr(), grad.data_ptr(), m.data_ptr(), v.data_ptr(), c, hgt * wid,
                                  float(lr), float(betas[0]), float(betas[1]), float(eps), int(step), int(clamp01), 1,
                                  _lib.stream_ptr(self.device)), "nst_adam_step")

    def run(self, content: torch.Tensor, style: torch.Tensor, steps: int = 300, lr: float = 0.02,
            content_weight: float = 1.0, style_weight: float = 1e6, init: Optional[torch.Tensor] = None,
            record_every: int = 0, trajectory: bool = False):
        """Optimise from `init` (default: the content image) for `steps` Adam updates.
        -> (image, list of (step, total, content, style) recorded every `record_every` steps); with
        `trajectory` every step's losses are kept on the device (no host synchronisation inside the loop) and
        returned as the list instead."""
        self.set_targets(content, style)
        x = (content if init is None else init).detach().to(self.device, torch.float32).clone().contiguous()
        m, v = torch.zeros_like(x), torch.zeros_like(x)
        hist = []
        g = torch.empty_like(x)
        losses = self.losses_for(x)
        traj = torch.empty((steps, 3), dtype=torch.float32, device=self.device) if trajectory else None
        sw = (1.0,) * 5
        for t in range(1, steps + 1):
            # the trajectory row is the losses buffer itself: no copy launch per step
            out = traj[t - 1] if trajectory else losses
            self._grad_into(x, g, out, content_weight, style_weight, sw)
            if not trajectory and record_every and (t == 1 or t % record_every == 0):
                hist.append((t - 1,) + tuple(float(z) for z in out[:3].cpu()))
            self.adam(x, g, m, v, t, lr)
        if traj is not None:
            hist = [(i,) + tuple(float(z) for z in row) for i, row in enumerate(traj.cpu())]
        return x, hist


def run_style_transfer(vgg_state: Dict[str, torch.Tensor], content: torch.Tensor, style: torch.Tensor,
                       num_steps: int = 300, style_weight: float = 1e6, content_weight: float = 1.0,
                       lr: float = 0.02, device: Optional[torch.device] = None) -> torch.Tensor:
    """The optimisation loop of configs[2] (Adam, `num_steps` updates, image clamped to [0, 1])."""
    dev = device or content.device
    g = Gatys(vgg_state, dev)
    out, _ = g.run(content.to(dev), style.to(dev), num_steps, lr, content_weight, style_weight)
    return out
