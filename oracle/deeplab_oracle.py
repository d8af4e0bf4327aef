"""CPU oracle for the DeepLab v3+ mask path (configs[4]) — TEST INFRASTRUCTURE ONLY.

Imported by tests/ (and tools/ benches' CPU legs) as the checker, never by neuralstyletransferv1_amd/.
Restates, in the reference's own arithmetic (PyTorch-CPU fp32 functional ops, numpy, Pillow):
  * forward(): modeling/deeplab.py:27-33 with backbone resnet.py:113-124 (Bottleneck :23-43), ASPP
    aspp.py:65-78, decoder decoder.py:34-43, BatchNorm2d in eval mode (sky_swap.py:160-176 builds
    DeepLab(sync_bn=False) and calls .eval()).  Pinned bit-exact against the reference modules by
    tests/golden/make_golden_deeplab.py (run in the build container with /root/reference).
  * preprocess_u8(): sky_swap.py:179-183 preprocess_pil.
  * infer_post(): sky_swap.py:189-215 (argmax, class OR, cv2 close / dilate / erode / GaussianBlur).
    cv2 is not importable here: the morphology is restated from OpenCV's definition (rectangular max /
    min over the window clipped to the image — binary masks make it unambiguous); the blur reuses
    nst_oracle.feather_mask_u8 (parity unpinned).
  * lanczos(): Pillow's Image.resize(LANCZOS) itself (the reference's dependency) — sky_swap.py:294-301.
  * cv_resize_linear_u8(): cv2.resize INTER_LINEAR on u8, OpenCV's fixed-point path restated
    (sky_swap.py:321-324; parity unpinned: cv2 absent).
"""
from __future__ import annotations

from typing import Dict, Sequence

import numpy as np
import torch
import torch.nn.functional as F

from oracle import nst_oracle

LAYERS = (3, 4, 23, 3)


def _bn(sd: Dict[str, torch.Tensor], pre: str, x: torch.Tensor) -> torch.Tensor:
    return F.batch_norm(x, sd[pre + ".running_mean"], sd[pre + ".running_var"], sd[pre + ".weight"], sd[pre + ".bias"],
                        False, 0.1, 1e-5)


def _bottleneck(sd, pre: str, x: torch.Tensor, stride: int, dilation: int, has_ds: bool) -> torch.Tensor:
    """resnet.py:23-43."""
    out = F.relu(_bn(sd, pre + ".bn1", F.conv2d(x, sd[pre + ".conv1.weight"])))
    out = F.relu(_bn(sd, pre + ".bn2", F.conv2d(out, sd[pre + ".conv2.weight"], stride=stride, padding=dilation,
                                                dilation=dilation)))
    out = _bn(sd, pre + ".bn3", F.conv2d(out, sd[pre + ".conv3.weight"]))
    residual = _bn(sd, pre + ".downsample.1", F.conv2d(x, sd[pre + ".downsample.0.weight"], stride=stride)) if has_ds else x
    out += residual
    return F.relu(out)


def backbone(sd, x: torch.Tensor):
    """resnet.py:113-124 at output stride 16 (strides 1,2,2,1; dilations 1,1,1,2; layer4 multi-grid 1,2,4)."""
    x = F.relu(_bn(sd, "backbone.bn1", F.conv2d(x, sd["backbone.conv1.weight"], stride=2, padding=3)))
    x = F.max_pool2d(x, 3, 2, 1)
    low = None
    for li, (nb, stride) in enumerate(zip(LAYERS, (1, 2, 2, 1))):
        for i in range(nb):
            dil = 1 if li < 3 else 2 * (1, 2, 4)[i]
            x = _bottleneck(sd, f"backbone.layer{li + 1}.{i}", x, stride if i == 0 else 1, dil, i == 0)
        if li == 0:
            low = x
    return x, low


def aspp(sd, x: torch.Tensor) -> torch.Tensor:
    """aspp.py:65-78 (dilations 1, 6, 12, 18; Dropout is the identity in eval)."""
    xs = []
    for i, d in enumerate((1, 6, 12, 18)):
        pre = f"aspp.aspp{i + 1}"
        pad = 0 if i == 0 else d
        xs.append(F.relu(_bn(sd, pre + ".bn", F.conv2d(x, sd[pre + ".atrous_conv.weight"], padding=pad, dilation=d))))
    x5 = F.adaptive_avg_pool2d(x, (1, 1))
    x5 = F.relu(_bn(sd, "aspp.global_avg_pool.2", F.conv2d(x5, sd["aspp.global_avg_pool.1.weight"])))
    x5 = F.interpolate(x5, size=xs[3].size()[2:], mode="bilinear", align_corners=True)
    x = torch.cat(xs + [x5], dim=1)
    return F.relu(_bn(sd, "aspp.bn1", F.conv2d(x, sd["aspp.conv1.weight"])))


def decoder(sd, x: torch.Tensor, low: torch.Tensor) -> torch.Tensor:
    """decoder.py:34-43."""
    low = F.relu(_bn(sd, "decoder.bn1", F.conv2d(low, sd["decoder.conv1.weight"])))
    x = F.interpolate(x, size=low.size()[2:], mode="bilinear", align_corners=True)
    x = torch.cat((x, low), dim=1)
    x = F.relu(_bn(sd, "decoder.last_conv.1", F.conv2d(x, sd["decoder.last_conv.0.weight"], padding=1)))
    x = F.relu(_bn(sd, "decoder.last_conv.5", F.conv2d(x, sd["decoder.last_conv.4.weight"], padding=1)))
    return F.conv2d(x, sd["decoder.last_conv.8.weight"], sd["decoder.last_conv.8.bias"])


@torch.no_grad()
def forward(sd: Dict[str, torch.Tensor], x: torch.Tensor) -> torch.Tensor:
    """deeplab.py:27-33: logits [n, nc, h, w]."""
    feat, low = backbone(sd, x)
    y = decoder(sd, aspp(sd, feat), low)
    return F.interpolate(y, size=x.size()[2:], mode="bilinear", align_corners=True)


def preprocess_u8(frame: np.ndarray) -> torch.Tensor:
    """sky_swap.py:179-183 on one uint8 HxWx3 RGB frame -> [1,3,h,w] fp32."""
    im = frame.astype(np.float32) / 255.0
    im = (im - (0.485, 0.456, 0.406)) / (0.229, 0.224, 0.225)
    return torch.from_numpy(im).permute(2, 0, 1).unsqueeze(0).float()


def _morph(m: np.ndarray, k: int, op: str) -> np.ndarray:
    """cv2.dilate / cv2.erode with np.ones((k, k)), anchor at the centre, default border (ignored)."""
    h, w = m.shape
    a = k // 2
    fn = np.maximum if op == "dilate" else np.minimum
    pad = 0 if op == "dilate" else 255
    p = np.full((h + 2 * a, w + 2 * a), pad, dtype=np.uint8)
    p[a:a + h, a:a + w] = m
    out = p[a:a + h, 0:w].copy()
    for dx in range(1, k):
        out = fn(out, p[a:a + h, dx:dx + w])
    rows = np.full((h + 2 * a, w), pad, dtype=np.uint8)
    rows[a:a + h] = out
    res = rows[0:h].copy()
    for dy in range(1, k):
        res = fn(res, rows[dy:dy + h])
    return res


def infer_post(pred: np.ndarray, target_ids: Sequence[int], expand_px: int = 0, contract_px: int = 0,
               feather_px: int = 3, close_ks: int = 5) -> np.ndarray:
    """sky_swap.py:196-215 on one class map (uint8 HxW)."""
    sky = np.zeros_like(pred, dtype=np.uint8)
    for cid in target_ids:
        sky |= (pred == int(cid)).astype(np.uint8)
    sky = (sky * 255).astype(np.uint8)
    if close_ks > 1:
        sky = _morph(_morph(sky, close_ks, "dilate"), close_ks, "erode")
    if int(expand_px) > 0:
        sky = _morph(sky, int(expand_px) * 2 + 1, "dilate")
    if int(contract_px) > 0:
        sky = _morph(sky, int(contract_px) * 2 + 1, "erode")
    if int(feather_px) > 0:
        sky = nst_oracle.feather_mask_u8(sky, int(feather_px))
    return sky


def lanczos(frame: np.ndarray, ow: int, oh: int) -> np.ndarray:
    """Pillow Image.resize((ow, oh), Image.LANCZOS) of an RGB uint8 frame (sky_swap.py:299)."""
    from PIL import Image
    return np.asarray(Image.fromarray(frame).resize((ow, oh), Image.LANCZOS))


def _cv_round_short(v: np.ndarray) -> np.ndarray:
    return np.clip(np.rint(v.astype(np.float64)), -32768, 32767).astype(np.int64)


def cv_resize_linear_u8(m: np.ndarray, ow: int, oh: int) -> np.ndarray:
    """cv2.resize(m, (ow, oh), interpolation=cv2.INTER_LINEAR) for uint8 HxW or HxWxC (OpenCV imgproc/resize.cpp
    fixed-point path: taps saturate_cast<short>(w * 2048); horizontal int sums; vertical
    (((b0 * (S0 >> 4)) >> 16) + ((b1 * (S1 >> 4)) >> 16) + 2) >> 2)."""
    src = m if m.ndim == 3 else m[..., None]
    h, w, c = src.shape

    def axis(n_in, n_out, clamp):
        scale = 1.0 / (n_out / n_in)
        d = np.arange(n_out, dtype=np.float64)
        f = ((d + 0.5) * scale - 0.5).astype(np.float32)
        s = np.floor(f).astype(np.int64)
        f = (f - s.astype(np.float32)).astype(np.float32)
        if clamp:
            lo = s < 0
            f[lo] = 0
            s[lo] = 0
            hi = s >= n_in - 1
            f[hi] = 0
            s[hi] = n_in - 1
        t0 = _cv_round_short((np.float32(1.0) - f) * np.float32(2048.0))
        t1 = _cv_round_short(f * np.float32(2048.0))
        return s, t0, t1

    sx, a0, a1 = axis(w, ow, True)
    sy, b0, b1 = axis(h, oh, False)
    sx1 = np.minimum(sx + 1, w - 1)
    x = src.astype(np.int64)
    hs = x[:, sx, :] * a0[None, :, None] + x[:, sx1, :] * a1[None, :, None]  # [h, ow, c]
    r0 = np.clip(sy, 0, h - 1)
    r1 = np.clip(sy + 1, 0, h - 1)
    S0, S1 = hs[r0], hs[r1]
    v = (((b0[:, None, None] * (S0 >> 4)) >> 16) + ((b1[:, None, None] * (S1 >> 4)) >> 16) + 2) >> 2
    out = np.clip(v, 0, 255).astype(np.uint8)
    return out if m.ndim == 3 else out[..., 0]


def masks_from_frames(sd, frames: np.ndarray, target_ids: Sequence[int], resolution: int = 256, expand_px: int = 0,
                      contract_px: int = 0, feather_px: int = 3):
    """batch_masks_from_frames (sky_swap.py:286-362) for in-memory frames: -> (masks [n,H,W], preds [n,h,w],
    logits [n,nc,h,w]) at the working size h x w."""
    masks, preds, logits = [], [], []
    for f in frames:
        H, W = f.shape[:2]
        w, h = W, H
        if resolution and resolution > 0:
            scale = float(resolution) / max(W, H)
            if scale < 1.0:
                w, h = int(W * scale), int(H * scale)
        work = f if (w, h) == (W, H) else lanczos(f, w, h)
        lg = forward(sd, preprocess_u8(work))
        pred = lg.argmax(1).squeeze(0).numpy().astype(np.uint8)
        m = infer_post(pred, target_ids, expand_px, contract_px, feather_px)
        if (w, h) != (W, H):
            m = cv_resize_linear_u8(m, W, H)
        masks.append(m)
        preds.append(pred)
        logits.append(lg[0].numpy())
    return np.stack(masks), np.stack(preds), np.stack(logits)
