"""Seeded synthetic checkpoints and frames (the reference's .pth weights are not shipped:
.MISSING_LARGE_BLOBS lists candy/mosaic/rain_princess/udnie/mosaic_reconet).

Weights come from numpy's PCG64 (portable across machines and torch versions) with the
reference's exact state_dict names/shapes, and are output-calibrated so the stylized
image spans the io_preset's range instead of collapsing to black:
  * every conv before an InstanceNorm: N(0, 2/fan_in); bias U(-0.05, 0.05)
  * InstanceNorm affine: gamma U(0.8, 1.2), beta U(-0.2, 0.2)
  * reconet_frn (ReCoNet(frn=True)): FRN weight U(0.8, 1.2), bias U(-0.2, 0.2), eps 1e-6 (seed 0) or
    -1e-3 (other seeds: |eps| is what FRN adds); TLU tau U(-0.3, 0.3)
  * the output conv: std chosen so the raw output has std ~TARGET_STD around TARGET_MEAN
    (Johnson raw/imagenet_255: 127.5 +- 60; NST raw_01: 0.5 +- 0.25; ReCoNet pre-tanh: 0 +- 1).
Frames: smooth gradients + shapes + low-amplitude noise so InstanceNorm statistics are
natural-image-like.
"""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch

ARCHS = ("johnson", "nst", "reconet", "reconet_frn")
_OUTPUT_CAL = {"johnson": (127.5, 60.0), "nst": (0.5, 0.25), "reconet": (0.0, 1.0), "reconet_frn": (0.0, 1.0)}
# raw-output calibration for a checkpoint trained with a given io_preset (pipeline.py:1445-1486 decodes): the raw
# output whose decode is ~0.5 +- 0.235 (the 127.5 +- 60 of the 0..255 presets), so the stylized frame spans the
# preset's range; channel means / stds of the ImageNet presets averaged over RGB
_PRESET_CAL = {
    "imagenet_255": (127.5, 60.0), "raw_255": (127.5, 60.0), "caffe_bgr": (127.5, 60.0),
    "raw_01": (0.5, 0.235), "tanh": (0.0, 0.47),
    "imagenet_01": ((0.5 - (0.485 + 0.456 + 0.406) / 3) / ((0.229 + 0.224 + 0.225) / 3), 0.235 / ((0.229 + 0.224 + 0.225) / 3)),
}


def build_module(arch: str):
    if arch == "johnson":
        from .transformer_net import TransformerNet
        return TransformerNet()
    if arch == "nst":
        from .transformer_net_nst import TransformerNet
        return TransformerNet()
    if arch in ("reconet", "reconet_frn"):
        from .model import ReCoNet
        return ReCoNet(frn=arch == "reconet_frn")
    raise ValueError(f"unknown arch {arch!r}")


def _final_conv_name(arch: str) -> str:
    return {"johnson": "deconv3.conv2d", "nst": "final", "reconet": "decoder.layers.4.layers.0.layers.1",
            "reconet_frn": "decoder.layers.4.layers.0.layers.1"}[arch]


def make_state_dict(arch: str, seed: int = 0, preset: str | None = None) -> Dict[str, torch.Tensor]:
    """Ordered {name: fp32 tensor} with the reference's keys for `arch`.  `preset` (Johnson): calibrate the output
    conv for a checkpoint trained with that io_preset (_PRESET_CAL); every other tensor is the same as without it
    (the random stream is consumed identically, only the output conv's scale and offset differ)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    template = build_module(arch).state_dict()
    final = _final_conv_name(arch)
    mean, std = _OUTPUT_CAL[arch] if preset is None else _PRESET_CAL[preset]
    out: Dict[str, torch.Tensor] = {}
    for name, t in template.items():
        shape = tuple(t.shape)
        if name == final + ".weight":
            fan_in = shape[1] * shape[2] * shape[3]
            v = rng.standard_normal(shape) * (std / np.sqrt(fan_in * 0.5))
        elif name == final + ".bias":
            v = mean + rng.uniform(-0.02, 0.02, shape) * max(std, 1e-3)
        elif name.endswith(".tau"):  # TLU threshold [1, C, 1, 1]
            v = rng.uniform(-0.3, 0.3, shape)
        elif name.endswith(".eps"):  # FRN eps buffer [1]
            v = np.full(shape, 1e-6 if seed == 0 else -1e-3)
        elif len(shape) == 4 and shape[0] == 1 and shape[2:] == (1, 1) and name.endswith(".weight"):  # FRN gamma
            v = rng.uniform(0.8, 1.2, shape)
        elif len(shape) == 4 and shape[0] == 1 and shape[2:] == (1, 1) and name.endswith(".bias"):  # FRN beta
            v = rng.uniform(-0.2, 0.2, shape)
        elif len(shape) == 4:
            # Conv2d [out,in,k,k]; ConvTranspose2d [in,out,k,k] (fan_in = out*k*k seen per output)
            fan_in = shape[1] * shape[2] * shape[3]
            v = rng.standard_normal(shape) * np.sqrt(2.0 / fan_in)
        elif name.endswith(".weight"):  # InstanceNorm gamma
            v = rng.uniform(0.8, 1.2, shape)
        elif name.endswith(".bias"):
            is_norm = name.rsplit(".", 1)[0] + ".weight" in template and template[name.rsplit(".", 1)[0] + ".weight"].dim() == 1
            v = rng.uniform(-0.2, 0.2, shape) if is_norm else rng.uniform(-0.05, 0.05, shape)
        else:
            v = np.zeros(shape)
        out[name] = torch.from_numpy(np.ascontiguousarray(v, dtype=np.float32))
    return out


def make_frames(n: int, h: int, w: int, seed: int = 0) -> np.ndarray:
    """uint8 [n,h,w,3] seeded natural-ish RGB frames."""
    rng = np.random.Generator(np.random.PCG64(seed))
    yy = np.linspace(0.0, 1.0, h, dtype=np.float32)[:, None]
    xx = np.linspace(0.0, 1.0, w, dtype=np.float32)[None, :]
    frames = np.empty((n, h, w, 3), dtype=np.uint8)
    for f in range(n):
        img = np.empty((h, w, 3), dtype=np.float32)
        for c in range(3):
            a, b, ph = rng.uniform(0.2, 1.0), rng.uniform(0.2, 1.0), rng.uniform(0, 2 * np.pi)
            img[..., c] = 0.5 + 0.35 * np.sin(2 * np.pi * (a * xx + b * yy) + ph)
        for _ in range(6):  # discs and boxes
            cy, cx = rng.uniform(0, 1, 2)
            r = rng.uniform(0.05, 0.25)
            col = rng.uniform(0, 1, 3).astype(np.float32)
            if rng.uniform() < 0.5:
                m = ((yy - cy) ** 2 + ((xx - cx) * (w / h)) ** 2) < r * r
            else:
                m = (np.abs(yy - cy) < r) & (np.abs(xx - cx) * (w / h) < r)
            img[m] = 0.6 * img[m] + 0.4 * col
        img += rng.normal(0.0, 0.02, (h, w, 3)).astype(np.float32)
        frames[f] = np.clip(img * 255.0, 0, 255).astype(np.uint8)
    return frames


# VGG-19 `features` convs up to conv5_1 (torchvision indices) for the Gatys loop (configs[2]); the
# ImageNet weights cannot be fetched offline, so seeded He-initialised weights stand in
VGG19_CONVS = ((0, 3, 64), (2, 64, 64), (5, 64, 128), (7, 128, 128), (10, 128, 256), (12, 256, 256),
               (14, 256, 256), (16, 256, 256), (19, 256, 512), (21, 512, 512), (23, 512, 512), (25, 512, 512),
               (28, 512, 512))


def make_vgg19_state_dict(seed: int = 0) -> Dict[str, torch.Tensor]:
    """{features.N.weight, features.N.bias} fp32, N(0, 2/fan_in) weights, small uniform biases."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out: Dict[str, torch.Tensor] = {}
    for idx, cin, cout in VGG19_CONVS:
        w = rng.standard_normal((cout, cin, 3, 3)) * np.sqrt(2.0 / (cin * 9))
        b = rng.uniform(-0.02, 0.02, cout)
        out[f"features.{idx}.weight"] = torch.from_numpy(np.ascontiguousarray(w, dtype=np.float32))
        out[f"features.{idx}.bias"] = torch.from_numpy(np.ascontiguousarray(b, dtype=np.float32))
    return out
