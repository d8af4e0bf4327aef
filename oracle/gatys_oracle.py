"""ORACLE -- TEST INFRASTRUCTURE ONLY (imported by tests/ alone, never by the product path).

torch-CPU fp32 restatement of the Gatys loop that libnst_hip's nst_vgg_* / nst_gatys_* /
nst_adam_step implement (configs[2]).  The reference has no VGG network, loss or optimiser
(SURVEY.md §0.3), only the two helpers this uses as written there:
  * gram_matrix          utils.py:80-83   (via nst_oracle.gram_matrix)
  * preprocess_for_vgg   utils.py:93-96   (ImageNet mean / std normalisation)
Everything else follows torch's own definitions: torchvision vgg19().features layers (Conv2d 3x3
pad 1 + ReLU, MaxPool2d(2)), F.mse_loss, autograd, torch.optim.Adam.  PARITY UNPINNED by the
reference (no loop to compare with); the GPU path is checked against this restatement.

bf16=True rounds where the engine stores bf16 (the weights, the normalised image, every conv's
pre-activation z) with straight-through gradients: the max-pool then sees the engine's ties, so
the gradient routing through each 2x2 window matches (in fp32 the window maximum can differ from
the bf16 one, which moves that window's gradient to another pixel: ~2 % of the routed positions
per pool layer on smooth images, the reason the fp32 comparison of gradients is looser).
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import torch
import torch.nn.functional as F

from . import nst_oracle as O

MEAN = torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)  # utils.py:93-96
STD = torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)
# (features index, pool after the ReLU) up to conv5_1
CONVS = ((0, False), (2, True), (5, False), (7, True), (10, False), (12, False), (14, False), (16, True),
         (19, False), (21, False), (23, False), (25, True), (28, False))
STYLE_IDX = (0, 5, 10, 19, 28)   # relu1_1 .. relu5_1
CONTENT_IDX = 21                 # relu4_2


def _rb(t: torch.Tensor) -> torch.Tensor:
    """bf16 rounding of the values, identity for the gradient."""
    return t + (t.to(torch.bfloat16).float() - t).detach()


def features(sd: Dict[str, torch.Tensor], x: torch.Tensor, pre_activation: bool = False,
             bf16: bool = False, keep_z: list = None) -> Dict[int, torch.Tensor]:
    """{features index: ReLU output (or the conv's pre-activation)} of the loss layers; keep_z
    (a list) receives every conv's z in order."""
    h = (x - MEAN) / STD
    if bf16:
        h = _rb(h)
    out = {}
    for idx, pool in CONVS:
        W = sd[f"features.{idx}.weight"]
        z = F.conv2d(h, W.to(torch.bfloat16).float() if bf16 else W, sd[f"features.{idx}.bias"], padding=1)
        if bf16:
            z = _rb(z)
        if keep_z is not None:
            if z.requires_grad:
                z.retain_grad()
            keep_z.append(z)
        a = F.relu(z)
        if idx in STYLE_IDX or idx == CONTENT_IDX:
            out[idx] = z if pre_activation else a
        h = F.max_pool2d(a, 2) if pool else a
    return out


def losses(sd, x, content, style, content_weight=1.0, style_weight=1e6, layer_weights: Sequence[float] = (1.0,) * 5,
           bf16: bool = False, keep_z: list = None):
    """-> (total, content, style) scalars with autograd through x."""
    with torch.no_grad():
        fs = features(sd, style, bf16=bf16)
        fc = features(sd, content, bf16=bf16)
        A = [O.gram_matrix(fs[i]) for i in STYLE_IDX]
        P = fc[CONTENT_IDX]
        if bf16:
            P = P.to(torch.bfloat16).float()
    fx = features(sd, x, bf16=bf16, keep_z=keep_z)
    lc = content_weight * F.mse_loss(fx[CONTENT_IDX], P)
    ls = style_weight * sum(w * F.mse_loss(O.gram_matrix(fx[i]), a) for i, a, w in zip(STYLE_IDX, A, layer_weights))
    return lc + ls, lc, ls


def run(sd, content, style, steps: int, lr: float, content_weight=1.0, style_weight=1e6) -> Tuple[torch.Tensor, List]:
    """Adam from the content image, clamped to [0, 1] after every update; -> (image, [(total, c, s)])."""
    x = content.clone().requires_grad_(True)
    opt = torch.optim.Adam([x], lr=lr)
    hist = []
    for _ in range(steps):
        opt.zero_grad()
        tot, lc, ls = losses(sd, x, content, style, content_weight, style_weight)
        tot.backward()
        hist.append((float(tot), float(lc), float(ls)))
        opt.step()
        with torch.no_grad():
            x.clamp_(0, 1)
    return x.detach(), hist
