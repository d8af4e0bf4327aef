"""DeepLab v3+ (ResNet-101, output stride 16) mask network — drop-in for the reference's
modeling/deeplab.py as sky_swap.py:143-177 `load_deeplab` builds it (backbone 'resnet', BatchNorm2d,
eval mode), plus the GPU mask path of sky_swap.py:185-219 `infer_mask` and :271-366
`batch_masks_from_frames` (BASELINE.json configs[4]).

`DeepLab` keeps the reference module's submodule names and parameter shapes
(backbone.layer3.22.conv2.weight, aspp.global_avg_pool.1.weight, decoder.last_conv.8.bias, ...), so a
`deeplab-resnet.pth.tar` state_dict loads unchanged; its parameters are containers only and `forward`
runs the network as libnst_hip kernels (csrc/seg_deeplab.cpp, csrc/conv_gemm.hip).  There is no CPU
path.  `MaskEngine` is the frame-batch API the stylization pipeline uses: frames in HBM ->
LANCZOS working-size downscale -> DeepLab -> argmax -> class selection -> close / expand / contract /
feather -> INTER_LINEAR upscale, all on the device.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Iterable, Optional, Sequence, Tuple

import numpy as np
import torch
from torch import nn

from . import _lib
from ._lib import NstError, NstParam, check, lib

_DTYPES = {"fp32": _lib.NST_DT_F32, "float32": _lib.NST_DT_F32, "bf16": _lib.NST_DT_BF16, "bfloat16": _lib.NST_DT_BF16,
           "fp16": _lib.NST_DT_F16, "float16": _lib.NST_DT_F16, "fp32s": _lib.NST_DT_F32S}

# resnet.py:153 ResNet101 blocks per layer; :50-56 output stride 16 strides / dilations; :50 multi-grid
RESNET101_LAYERS = (3, 4, 23)
MULTI_GRID = (1, 2, 4)


def _bn(c: int) -> nn.BatchNorm2d:
    return nn.BatchNorm2d(c)


class Bottleneck(nn.Module):
    """resnet.py:6-43 (expansion 4; stride and dilation on the 3x3)."""

    def __init__(self, inplanes: int, planes: int, stride: int = 1, dilation: int = 1, downsample: bool = False):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = _bn(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, dilation=dilation, padding=dilation, bias=False)
        self.bn2 = _bn(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = _bn(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = (nn.Sequential(nn.Conv2d(inplanes, planes * 4, 1, stride=stride, bias=False), _bn(planes * 4))
                           if downsample else None)


class ResNet(nn.Module):
    """resnet.py:45-124 with output_stride=16 (strides 1,2,2,1; dilations 1,1,1,2; multi-grid layer4)."""

    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = _bn(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        inplanes = 64
        for li, (planes, stride) in enumerate(((64, 1), (128, 2), (256, 2), (512, 1))):
            if li < 3:
                dil = [1] * RESNET101_LAYERS[li]
            else:
                dil = [2 * g for g in MULTI_GRID]
            blocks = []
            for i, d in enumerate(dil):
                blocks.append(Bottleneck(inplanes, planes, stride if i == 0 else 1, d, downsample=(i == 0)))
                inplanes = planes * 4
            setattr(self, f"layer{li + 1}", nn.Sequential(*blocks))


class _ASPPModule(nn.Module):
    """aspp.py:7-21."""

    def __init__(self, inplanes: int, planes: int, kernel_size: int, padding: int, dilation: int):
        super().__init__()
        self.atrous_conv = nn.Conv2d(inplanes, planes, kernel_size, stride=1, padding=padding, dilation=dilation,
                                     bias=False)
        self.bn = _bn(planes)
        self.relu = nn.ReLU()


class ASPP(nn.Module):
    """aspp.py:34-78 for the resnet backbone at output stride 16 (dilations 1, 6, 12, 18)."""

    def __init__(self):
        super().__init__()
        for i, d in enumerate((1, 6, 12, 18)):
            k = 1 if d == 1 else 3
            setattr(self, f"aspp{i + 1}", _ASPPModule(2048, 256, k, 0 if k == 1 else d, d))
        self.global_avg_pool = nn.Sequential(nn.AdaptiveAvgPool2d((1, 1)), nn.Conv2d(2048, 256, 1, stride=1, bias=False),
                                             _bn(256), nn.ReLU())
        self.conv1 = nn.Conv2d(1280, 256, 1, bias=False)
        self.bn1 = _bn(256)
        self.relu = nn.ReLU()
        self.dropout = nn.Dropout(0.5)


class Decoder(nn.Module):
    """decoder.py:7-43 (resnet: 256 low-level channels)."""

    def __init__(self, num_classes: int):
        super().__init__()
        self.conv1 = nn.Conv2d(256, 48, 1, bias=False)
        self.bn1 = _bn(48)
        self.relu = nn.ReLU()
        self.last_conv = nn.Sequential(
            nn.Conv2d(304, 256, 3, stride=1, padding=1, bias=False), _bn(256), nn.ReLU(), nn.Dropout(0.5),
            nn.Conv2d(256, 256, 3, stride=1, padding=1, bias=False), _bn(256), nn.ReLU(), nn.Dropout(0.1),
            nn.Conv2d(256, num_classes, 1, stride=1))


class SegEngine:
    """One packed DeepLab checkpoint on one device (owns an nst_seg handle and a workspace)."""

    def __init__(self, state: Dict[str, torch.Tensor], num_classes: int, dtype: str, device: torch.device):
        if device.type != "cuda":
            raise NstError("libnst_hip runs on MI355X (cuda) devices only; there is no CPU path")
        if dtype not in _DTYPES:
            raise NstError(f"compute_dtype must be fp32, fp32s, bf16 or fp16, got {dtype!r}")
        self.device = device
        self.num_classes = int(num_classes)
        self.dtype = _DTYPES[dtype]
        host = {k: v.detach().to("cpu", torch.float32).contiguous() for k, v in state.items()
                if v.is_floating_point()}
        names = list(host)
        arr = (NstParam * len(names))()
        keep = []
        for i, k in enumerate(names):
            b = k.encode()
            keep.append(b)
            arr[i].name = b
            arr[i].data = ctypes.cast(host[k].data_ptr(), ctypes.POINTER(ctypes.c_float))
            arr[i].numel = host[k].numel()
        h = ctypes.c_void_p()
        dev_index = device.index if device.index is not None else torch.cuda.current_device()
        check(lib().nst_seg_create(arr, len(names), self.num_classes, self.dtype, dev_index, ctypes.byref(h)),
              "nst_seg_create")
        self._h = h
        self._ws: Optional[torch.Tensor] = None

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().nst_seg_destroy(h)
            except Exception:
                pass
            self._h = None

    def workspace(self, n: int, h: int, w: int) -> torch.Tensor:
        need = ctypes.c_size_t()
        check(lib().nst_seg_workspace_bytes(self._h, n, h, w, ctypes.byref(need)), "nst_seg_workspace_bytes")
        if self._ws is None or self._ws.numel() < need.value:
            self._ws = torch.empty(max(need.value, 256), dtype=torch.uint8, device=self.device)
        self._ws.record_stream(torch.cuda.current_stream(self.device))
        return self._ws

    def run(self, x: torch.Tensor, logits: bool = True, pred: bool = False):
        """x: module input f32 [n,3,h,w] or frames u8 [n,h,w,3] (preprocess_pil fused).
        -> (logits f32 [n,nc,h,w] or None, pred u8 [n,h,w] or None)."""
        _lib.require_gpu_tensor(x, "input")
        x = x.contiguous()
        if x.dtype == torch.uint8:
            if x.dim() != 4 or x.shape[3] != 3:
                raise NstError(f"expected uint8 [N,H,W,3] frames, got {tuple(x.shape)}")
            n, h, w, _ = x.shape
            fmt = _lib.NST_IO_U8_NHWC
        else:
            if x.dim() != 4 or x.shape[1] != 3:
                raise NstError(f"expected [N,3,H,W] input, got {tuple(x.shape)}")
            x = x.to(torch.float32)
            n, _, h, w = x.shape
            fmt = _lib.NST_IO_F32_NCHW
        lg = torch.empty((n, self.num_classes, h, w), dtype=torch.float32, device=self.device) if logits else None
        pr = torch.empty((n, h, w), dtype=torch.uint8, device=self.device) if pred else None
        ws = self.workspace(n, h, w)
        check(lib().nst_seg_forward(self._h, x.data_ptr(), fmt, n, h, w, lg.data_ptr() if lg is not None else None,
                                    pr.data_ptr() if pr is not None else None, ws.data_ptr(), ws.numel(),
                                    _lib.stream_ptr(self.device)), "nst_seg_forward")
        return lg, pr


class DeepLab(nn.Module):
    """modeling/deeplab.py:9-33 with backbone='resnet', output_stride=16, sync_bn=False (sky_swap.py:160-166)."""

    def __init__(self, backbone: str = "resnet", output_stride: int = 16, num_classes: int = 21, sync_bn: bool = True,
                 freeze_bn: bool = False):
        super().__init__()
        if backbone != "resnet" or output_stride != 16:
            raise NstError("libnst_hip builds DeepLab v3+ with backbone='resnet', output_stride=16 "
                           "(what sky_swap.py load_deeplab uses)")
        self.num_classes = int(num_classes)
        self.backbone = ResNet()
        self.aspp = ASPP()
        self.decoder = Decoder(num_classes)
        self.freeze_bn = freeze_bn
        self.compute_dtype = "fp32"
        self._engines: Dict[Tuple[int, str], Tuple[tuple, SegEngine]] = {}

    def _param_key(self) -> tuple:
        return tuple((t.data_ptr(), t._version) for t in self.state_dict().values())

    def engine(self, device: Optional[torch.device] = None, dtype: Optional[str] = None) -> SegEngine:
        if device is None:
            device = next(self.parameters()).device
        device = torch.device(device)
        if device.type != "cuda":
            raise NstError("move the module (or pass a device) to an MI355X first: there is no CPU path")
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        dtype = dtype or self.compute_dtype
        key = (device.index, dtype)
        pk = self._param_key()
        hit = self._engines.get(key)
        if hit is not None and hit[0] == pk:
            return hit[1]
        eng = SegEngine(self.state_dict(), self.num_classes, dtype, device)
        self._engines[key] = (pk, eng)
        return eng

    def forward(self, input: torch.Tensor) -> torch.Tensor:  # noqa: A002 (reference signature)
        _lib.require_gpu_tensor(input, "input")
        return self.engine(input.device).run(input, logits=True, pred=False)[0]

    def _apply(self, fn, *args, **kwargs):
        self._engines = {}
        return super()._apply(fn, *args, **kwargs)


class Resampler:
    """One nst_resize geometry: kind "lanczos" (PIL Image.resize LANCZOS, RGB) or "cv_linear"
    (cv2.resize INTER_LINEAR, any channel count)."""

    KINDS = {"lanczos": 0, "cv_linear": 1}

    def __init__(self, kind: str, h: int, w: int, oh: int, ow: int, device: torch.device):
        self.kind, self.h, self.w, self.oh, self.ow, self.device = kind, h, w, oh, ow, device
        r = ctypes.c_void_p()
        check(lib().nst_resize_create(self.KINDS[kind], h, w, oh, ow, device.index or 0, ctypes.byref(r)),
              "nst_resize_create")
        self._r = r

    def __del__(self):
        r = getattr(self, "_r", None)
        if r is not None and r.value:
            try:
                lib().nst_resize_destroy(r)
            except Exception:
                pass
            self._r = None

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        """x: u8 [n,h,w] or [n,h,w,c] -> same layout at (oh, ow)."""
        _lib.require_gpu_tensor(x, "image")
        if x.dtype != torch.uint8 or x.shape[1:3] != (self.h, self.w):
            raise NstError(f"expected uint8 [N,{self.h},{self.w}(,C)] images, got {x.dtype} {tuple(x.shape)}")
        x = x.contiguous()
        c = x.shape[3] if x.dim() == 4 else 1
        n = x.shape[0]
        out = torch.empty((n, self.oh, self.ow) + ((c,) if x.dim() == 4 else ()), dtype=torch.uint8,
                          device=self.device)
        need = ctypes.c_size_t()
        check(lib().nst_resize_scratch_bytes(self._r, n, ctypes.byref(need)), "nst_resize_scratch_bytes")
        scratch = torch.empty(max(need.value, 1), dtype=torch.uint8, device=self.device)
        check(lib().nst_resize_u8(self._r, x.data_ptr(), n, c, out.data_ptr(), scratch.data_ptr(), scratch.numel(),
                                  _lib.stream_ptr(self.device)), "nst_resize_u8")
        return out


def pct_to_px(pct: float, base: int) -> int:
    """sky_swap.py:36-40 _pct_to_px_val."""
    try:
        return int(round(max(0.0, float(pct)) * 0.01 * base))
    except Exception:
        return 0


def working_size(w: int, h: int, resolution: int) -> Tuple[int, int]:
    """sky_swap.py:294-299: downscale so the longer side is `resolution` (never upscale)."""
    if resolution and resolution > 0:
        scale = float(resolution) / max(w, h)
        if scale < 1.0:
            return int(w * scale), int(h * scale)
    return w, h


def mask_from_pred(pred: torch.Tensor, target_ids: Sequence[int], close_ks: int = 5, expand_px: int = 0,
                   contract_px: int = 0, feather_px: int = 3) -> torch.Tensor:
    """sky_swap.py:196-215 on class maps u8 [n,h,w] -> masks u8 [n,h,w]."""
    _lib.require_gpu_tensor(pred, "pred")
    pred = pred.contiguous()
    n, h, w = pred.shape
    ids = (ctypes.c_int * len(target_ids))(*[int(i) for i in target_ids])
    need = ctypes.c_size_t()
    check(lib().nst_seg_mask_scratch_bytes(n, h, w, ctypes.byref(need)), "nst_seg_mask_scratch_bytes")
    scratch = torch.empty(need.value, dtype=torch.uint8, device=pred.device)
    mask = torch.empty_like(pred)
    check(lib().nst_seg_mask(pred.data_ptr(), n, h, w, ids, len(target_ids), int(close_ks), int(expand_px),
                             int(contract_px), int(feather_px), mask.data_ptr(), scratch.data_ptr(), scratch.numel(),
                             _lib.stream_ptr(pred.device)), "nst_seg_mask")
    return mask


class MaskEngine:
    """Frames in HBM -> per-frame masks at frame size (sky_swap.py:271-366 batch_masks_from_frames for one
    batch, minus the PNG I/O): LANCZOS downscale to `resolution` on the longer side, DeepLab, argmax,
    target-id selection, close 5x5, expand / contract / feather (px or percent of the working height),
    INTER_LINEAR upscale back to the frame size."""

    def __init__(self, model: DeepLab, device: torch.device, resolution: int = 256, dtype: Optional[str] = None):
        self.model = model
        self.device = torch.device(device)
        self.resolution = int(resolution or 0)
        self.dtype = dtype
        self._rs: Dict[tuple, Resampler] = {}

    def _resampler(self, kind, h, w, oh, ow) -> Resampler:
        key = (kind, h, w, oh, ow)
        if key not in self._rs:
            self._rs[key] = Resampler(kind, h, w, oh, ow, self.device)
        return self._rs[key]

    def masks(self, frames: torch.Tensor, target_ids: Iterable[int], expand_px: int = 0, contract_px: int = 0,
              feather_px: int = 3, expand_pct: float = 0.0, contract_pct: float = 0.0, feather_pct: float = 0.0,
              close_ks: int = 5, return_pred: bool = False):
        _lib.require_gpu_tensor(frames, "frames")
        n, H, W, _ = frames.shape
        ww, hh = working_size(W, H, self.resolution)
        work = frames if (ww, hh) == (W, H) else self._resampler("lanczos", H, W, hh, ww)(frames)
        e_px = pct_to_px(expand_pct, hh) if expand_pct and expand_pct > 0 else int(expand_px)
        c_px = pct_to_px(contract_pct, hh) if contract_pct and contract_pct > 0 else int(contract_px)
        f_px = pct_to_px(feather_pct, hh) if feather_pct and feather_pct > 0 else int(feather_px)
        _, pred = self.model.engine(self.device, self.dtype).run(work, logits=False, pred=True)
        m = mask_from_pred(pred, list(target_ids), close_ks, e_px, c_px, f_px)
        if (ww, hh) != (W, H):
            m = self._resampler("cv_linear", hh, ww, H, W)(m)
        return (m, pred) if return_pred else m


# ---- label tables (sky_swap.py:83-122) ----
CITYSCAPES_SKY_ID_DEFAULT = 10
VOC21_LABELS = {n: i for i, n in enumerate((
    "background", "aeroplane", "bicycle", "bird", "boat", "bottle", "bus", "car", "cat", "chair", "cow",
    "diningtable", "dog", "horse", "motorbike", "person", "pottedplant", "sheep", "sofa", "train", "tvmonitor"))}
CITYSCAPES19_LABELS = {n: i for i, n in enumerate((
    "road", "sidewalk", "building", "wall", "fence", "pole", "traffic light", "traffic sign", "vegetation",
    "terrain", "sky", "person", "rider", "car", "truck", "bus", "train", "motorcycle", "bicycle"))}


def lookup_label_ids(label_names, used_nc: int):
    """sky_swap.py:105-122."""
    if used_nc == 21:
        table = VOC21_LABELS
    elif used_nc == 19:
        table = CITYSCAPES19_LABELS
    else:
        table = {**VOC21_LABELS, **CITYSCAPES19_LABELS}
    ids = []
    for name in label_names:
        key = name.strip().lower().replace("_", " ").replace("-", " ")
        if key in table:
            ids.append(int(table[key]))
        else:
            print(f"[warn] unknown label '{name}' for used_nc={used_nc}; skipping")
    return sorted(set(ids))


def detect_num_classes(state: Dict[str, torch.Tensor]) -> Optional[int]:
    """sky_swap.py:128-141: class count from the 1x1 conv weights (19/21/150/80 preferred)."""
    cand = []
    for v in state.values():
        if isinstance(v, torch.Tensor) and v.ndim == 4 and v.shape[2] == 1 and v.shape[3] == 1:
            k = int(v.shape[0])
            if 2 <= k <= 256:
                cand.append(k)
    for pref in (19, 21, 150, 80):
        if pref in cand:
            return pref
    return max(cand) if cand else None


def load_deeplab(weights_path: str, num_classes: Optional[int] = None, device="cuda", dtype: str = "bf16"):
    """sky_swap.py:143-177: checkpoint (optionally {"state_dict": ...}, "module." prefixes stripped), class count
    sniffed from the 1x1 convs, load_state_dict(strict=False).  Loaded with weights_only=True."""
    ckpt = torch.load(weights_path, map_location="cpu", weights_only=True)
    state = ckpt["state_dict"] if isinstance(ckpt, dict) and "state_dict" in ckpt else ckpt
    state = {k.replace("module.", "", 1): v for k, v in state.items()}
    detected = detect_num_classes(state)
    nc = num_classes if num_classes is not None else (detected if detected is not None else 19)
    print(f"[info] using num_classes={nc} (detected={detected}) backbone=resnet")
    model = DeepLab(num_classes=nc, backbone="resnet", output_stride=16, sync_bn=False, freeze_bn=False)
    missing, unexpected = model.load_state_dict(state, strict=False)
    if missing or unexpected:
        print(f"[warn] load_state: missing={len(missing)} unexpected={len(unexpected)}")
    model.compute_dtype = dtype
    return model.eval().to(device), int(nc)


def make_state_dict(num_classes: int = 19, seed: int = 0) -> Dict[str, torch.Tensor]:
    """Seeded synthetic DeepLab checkpoint with the reference's keys (the .pth.tar is not shipped:
    .gitignore:12-13).  numpy PCG64; convs N(0, 2/fan_in); BatchNorm gamma U(0.5, 1), beta U(-0.1, 0.1),
    running_mean U(-0.1, 0.1), running_var U(0.5, 1.5); each bottleneck's bn3 gamma U(0.1, 0.3) so the
    residual stream stays O(1) over 33 blocks; classifier N(0, 1/fan_in) with zero-sum rows, bias U(-0.1, 0.1)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    template = DeepLab(num_classes=num_classes).state_dict()
    out: Dict[str, torch.Tensor] = {}
    for name, t in template.items():
        shape = tuple(t.shape)
        if name.endswith("num_batches_tracked"):
            out[name] = torch.zeros((), dtype=torch.long)
            continue
        if len(shape) == 4:
            fan_in = shape[1] * shape[2] * shape[3]
            std = np.sqrt((1.0 if name.startswith("decoder.last_conv.8") else 2.0) / fan_in)
            v = rng.standard_normal(shape, dtype=np.float32) * np.float32(std)
            if name == "decoder.last_conv.8.weight":  # zero-sum rows: classes follow feature variation, not the
                v = v - v.mean(axis=1, keepdims=True)  # (shared, positive) post-ReLU feature mean
        elif name == "decoder.last_conv.8.bias":
            v = rng.uniform(-0.1, 0.1, shape)
        elif name.endswith("running_mean"):
            v = rng.uniform(-0.1, 0.1, shape)
        elif name.endswith("running_var"):
            v = rng.uniform(0.5, 1.5, shape)
        elif name.endswith(".weight"):
            v = rng.uniform(0.1, 0.3, shape) if ".bn3." in name else rng.uniform(0.5, 1.0, shape)
        elif name.endswith(".bias"):
            v = rng.uniform(-0.1, 0.1, shape)
        else:
            raise ValueError(name)
        out[name] = torch.from_numpy(np.ascontiguousarray(v, dtype=np.float32))
    return out
