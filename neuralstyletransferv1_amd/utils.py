"""Drop-in for the Gram / VGG-normalisation helpers of the reference's utils.py (:80-96).

`gram_matrix` runs on MFMA through libnst_hip (nst_gram); inputs must live on an MI355X.
"""
from __future__ import annotations

import torch

from . import _lib
from ._lib import check, lib

VGG_MEAN = (0.485, 0.456, 0.406)
VGG_STD = (0.229, 0.224, 0.225)


def gram_matrix(feature_map: torch.Tensor) -> torch.Tensor:
    """utils.py:80-83: G = F F^T / (c*h*w) per batch element; fp32 result."""
    _lib.require_gpu_tensor(feature_map, "feature_map")
    n, c, h, w = feature_map.shape
    if feature_map.dtype == torch.bfloat16:
        dt = _lib.NST_DT_BF16
    else:
        feature_map = feature_map.to(torch.float32)
        dt = _lib.NST_DT_F32
    f = feature_map.contiguous()
    return gram_raw(f, dt, _lib.NST_GRAM_CHW, n, c, h * w)


def gram_raw(f: torch.Tensor, dt: int, layout: int, n: int, c: int, hw: int) -> torch.Tensor:
    """nst_gram on a contiguous device buffer (CHW or HWC per batch element) -> [n,c,c] fp32."""
    import ctypes
    G = torch.empty((n, c, c), dtype=torch.float32, device=f.device)
    need = ctypes.c_size_t()
    check(lib().nst_gram_workspace_bytes(n, c, hw, ctypes.byref(need)), "nst_gram_workspace_bytes")
    ws = torch.empty(max(need.value, 16), dtype=torch.uint8, device=f.device)
    check(lib().nst_gram(f.data_ptr(), dt, layout, n, c, hw, G.data_ptr(), ws.data_ptr(), ws.numel(),
                         _lib.stream_ptr(f.device)), "nst_gram")
    return G


def normalize_batch(batch: torch.Tensor, mean, std) -> torch.Tensor:
    """utils.py:86-90 (elementwise, on the batch's device)."""
    mean = torch.as_tensor(mean, dtype=batch.dtype, device=batch.device)
    std = torch.as_tensor(std, dtype=batch.dtype, device=batch.device)
    return (batch - mean[None, :, None, None]) / std[None, :, None, None]


def preprocess_for_vgg(images_batch: torch.Tensor) -> torch.Tensor:
    """utils.py:93-96."""
    return normalize_batch(images_batch, mean=list(VGG_MEAN), std=list(VGG_STD))
