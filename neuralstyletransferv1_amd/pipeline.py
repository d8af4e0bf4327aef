#!/usr/bin/env python3
"""pipeline.py — drop-in for the reference's CLI (pipeline.py:2156-2671) on the MI355X engine.

Same flags, defaults and modes (single image / batch images / video) as the reference; the
per-frame loop (`style_frames`, pipeline.py:527-2122, standard path :1409-1519 + post chain
:1881-2119) runs batched on the GPU:

    host: PIL decode (thread pool) -> uint8 frames --H2D--> [GPU] preset encode + net forward +
    decode + clamp + ToPILImage truncation (one nst_forward per model slot) -> multi-model blend
    -> LAB EMA (LUT, frame order) -> mask composite -> uniform blend --D2H--> host: PIL encode.

Additions: --gpus N (frames round-robin over N GPUs, ordered gather to rank 0 over RCCL),
--batch B (frames per GPU step), --dtype {fp32,fp32s,fp16m,bf16,fp16} (fp32 = parity with the reference's
arithmetic, default; fp32s = fp32 activations on split-fp16 MFMAs, the parity bar at several times
fp32's speed; fp16m = split-fp16 on the layers whose rounding reaches the frame, fp16 elsewhere: +-1 LSB
at most of the fp16 rate; bf16 = throughput mode; fp16 = near bf16's speed with 3 more mantissa bits),
--synthetic WxH / --synthetic_frames N (an
in-memory synthetic frame stream instead of files; config 4 of BASELINE.json).

Also on the GPU: the LAB multi-model blend (--blend_models_lab, pipeline.py:1841-1870) and the
Gaussian mask feather (--mask_feather / --mask_feather_pct, pipeline.py:349-351; cv2's blur
restated, parity unpinned because cv2 is absent here).

Region blending (--region_mode / --region_optimize and their spec, animation and rotation flags,
pipeline.py:1120-1407, 1720-1839) runs on the GPU compositor of regions.py.

The flow-guided EMA (--flow_ema with --flow_method dis, the default, or farneback, pipeline.py:1884-1940; any
--flow_downscale factor, floored like the reference's (W0 // ds, H0 // ds)) and the motion-adaptive blend
(--motion_blend, :2072-2086) run on the GPU (temporal.py).

Not built (rejected with a clear message if requested): Magenta (TF-Hub) and Torch7
(OpenCV DNN) backends.
"""
from __future__ import annotations

import argparse
import glob
import os
import re
import shutil
import subprocess
import sys
import time
import uuid
from concurrent.futures import ThreadPoolExecutor
from datetime import timedelta
from pathlib import Path
from typing import Dict, List, Optional

import numpy as np

IO_PRESETS_AUTO = {  # pipeline.py:2518-2523
    "transformer": "imagenet_255",
    "torch7": "caffe_bgr",
    "magenta": "imagenet_01",
    "reconet": "imagenet_01",
}
SLOTS = ["b", "c", "d", "e", "f", "g", "h"]


# the last style_frames run on this process: frames, seconds of the frame loop (decode -> GPU -> encode, from the
# first frame load to the last file written) and seconds of setup before it (model load, plans, size scan)
LAST_RUN_STATS: Dict[str, float] = {}


def _log(msg: str) -> None:
    print(msg, flush=True)


# ----------------------------------------------------------------------------- argparse
def build_parser() -> argparse.ArgumentParser:
    """Flag-for-flag mirror of pipeline.py:2157-2410 (+ engine flags at the end)."""
    ap = argparse.ArgumentParser(description="Extract -> Style -> Assemble (with temporal smoothing) on MI355X")
    ap.add_argument("--input_video", default=None)
    ap.add_argument("--output_video", default=None)
    ap.add_argument("--model", required=False)
    ap.add_argument("--work_dir", default="./_work")
    ap.add_argument("--fps", type=int, default=None)
    ap.add_argument("--pre_fps", type=int, default=None)
    ap.add_argument("--scale", type=int, default=None)
    ap.add_argument("--canvas", type=str, default=None)
    ap.add_argument("--image_ext", choices=["png", "jpg"], default="png")
    ap.add_argument("--jpeg_quality", type=int, default=85)
    ap.add_argument("--threads", type=int, default=4, help="host threads for frame decode/encode")
    ap.add_argument("--stride", type=int, default=1)
    ap.add_argument("--max_frames", type=int, default=None)
    ap.add_argument("--device", choices=["cpu", "mps", "cuda"], default="cuda")
    ap.add_argument("--gpu_memory_limit", type=int, default=32000)
    ap.add_argument("--inference_res", type=int, default=0)
    ap.add_argument("--io_preset", choices=["auto", "imagenet_255", "imagenet_01", "tanh", "caffe_bgr", "raw_255", "raw_01"],
                    default="auto")
    ap.add_argument("--input_image", type=str)
    ap.add_argument("--output_image", type=str)
    ap.add_argument("--input_dir", type=str)
    ap.add_argument("--output_dir", type=str)
    ap.add_argument("--pattern", type=str, default=None)
    ap.add_argument("--keep_ext", action="store_true")
    ap.add_argument("--output_suffix", type=str, default="")
    ap.add_argument("--output_prefix", type=str, default="styled_frame")
    ap.add_argument("--smooth_lightness", action="store_true", default=True)
    ap.add_argument("--no-smooth_lightness", action="store_false", dest="smooth_lightness")
    ap.add_argument("--smooth_alpha", type=float, default=0.7)
    ap.add_argument("--smooth_chroma", action="store_true", default=False)
    ap.add_argument("--chroma_alpha", type=float, default=0.85)
    ap.add_argument("--blend", type=float, default=1.0)
    ap.add_argument("--mask", type=str, default=None)
    ap.add_argument("--mask_invert", action="store_true")
    ap.add_argument("--mask_feather", type=int, default=0)
    ap.add_argument("--mask_dir", type=str, default=None)
    ap.add_argument("--mask_feather_pct", type=float, default=0.0)
    ap.add_argument("--mask_autofix", action="store_true", default=True)
    ap.add_argument("--mask_force_transpose", action="store_true")
    ap.add_argument("--mask_debug_overlay", action="store_true")
    ap.add_argument("--mask_debug_alpha", action="store_true")
    ap.add_argument("--fit_mask_to", choices=["input", "output"], default="input")
    ap.add_argument("--composite_mode", choices=["keep", "replace"], default="keep")
    ap.add_argument("--flow_ema", action="store_true", default=False)
    ap.add_argument("--flow_alpha", type=float, default=0.85)
    ap.add_argument("--flow_method", choices=["farneback", "dis"], default="dis")
    ap.add_argument("--flow_downscale", type=int, default=1)
    ap.add_argument("--model_type", choices=["transformer", "reconet", "magenta", "torch7"], default="transformer")
    for s in SLOTS:
        ap.add_argument(f"--model_{s}", type=str, default=None)
        ap.add_argument(f"--model_{s}_type", choices=["transformer", "reconet", "magenta", "torch7"], default=None)
        ap.add_argument(f"--io_preset_{s}", choices=["imagenet_255", "imagenet_01", "tanh", "caffe_bgr", "raw_255", "raw_01"],
                        default=None)
        ap.add_argument(f"--magenta_style_{s}", type=str, default=None)
    ap.add_argument("--blend_models_weights", type=str, default=None)
    ap.add_argument("--blend_models_lab", action="store_true")
    ap.add_argument("--blend_models_lab_weights", type=str, default=None)
    for flag, kw in (("--region_mode", dict(type=str, default=None, choices=["grid", "diagonal", "voronoi", "fractal",
                                                                           "radial", "waves", "spiral", "concentric",
                                                                           "random"])),
                     ("--region_count", dict(type=int, default=None)),
                     ("--region_sizes", dict(type=str, default=None)), ("--region_seed", dict(type=str, default=None)),
                     ("--region_feather", dict(type=int, default=20)),
                     ("--region_assignment", dict(type=str, default="random", choices=["sequential", "random", "weighted"])),
                     ("--region_original", dict(type=float, default=0.0)), ("--region_rotate", dict(type=float, default=0.0)),
                     ("--region_blend_spec", dict(type=str, default=None)), ("--region_scales", dict(type=str, default=None)),
                     ("--region_optimize", dict(action="store_true")), ("--region_padding", dict(type=int, default=64)),
                     ("--blend_animate", dict(type=str, default=None)), ("--blend_animate_regions", dict(type=str, default=None)),
                     ("--scale_animate", dict(type=str, default=None)), ("--scale_animate_regions", dict(type=str, default=None)),
                     ("--region_morph", dict(type=str, default=None))):
        ap.add_argument(flag, **kw)
    ap.add_argument("--magenta_style", type=str, default=None)
    ap.add_argument("--magenta_model_root", type=str, default="/app/models/magenta")
    ap.add_argument("--magenta_tile", type=int, default=256)
    ap.add_argument("--magenta_overlap", type=int, default=32)
    ap.add_argument("--magenta_target_res", type=int, default=None)
    ap.add_argument("--motion_blend", action="store_true")
    ap.add_argument("--clean_frames", action="store_true")
    ap.add_argument("--clean_work_dir", action="store_true")
    # ---- engine flags ----
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("GPUS", "1")),
                    help="frames round-robin over N GPUs (one process per GPU), ordered gather to rank 0")
    ap.add_argument("--batch", type=int, default=8, help="frames per GPU per step")
    ap.add_argument("--dist_backend", choices=["nccl", "gloo"], default="nccl",
                    help="--gpus > 1 process group: nccl (RCCL over xGMI, one GPU per rank) or gloo (host-staged "
                         "exchange; ranks may share a GPU, used by the tests)")
    ap.add_argument("--dist_timeout", type=float, default=600.0, help="seconds before a blocked exchange aborts")
    ap.add_argument("--dtype", choices=["fp32", "fp32s", "fp16m", "bf16", "fp16"], default="fp32",
                    help="fp32 = parity with the reference arithmetic; fp32s = fp32 activations on split-fp16 "
                         "MFMAs (the same +-1 LSB parity, faster; conv inputs < 65504); fp16m = split-fp16 on the "
                         "first layers, fp16 elsewhere (+-1 LSB on 1080p frames, most of fp16's speed; ReCoNet runs "
                         "fp32s); bf16 = throughput mode; "
                         "fp16 = near the throughput mode's speed with 3 more mantissa bits (activations < 65504)")
    ap.add_argument("--synthetic", type=str, default=None, help="WxH: stylize an in-memory synthetic frame stream")
    ap.add_argument("--synthetic_frames", type=int, default=16)
    ap.add_argument("--no_save", action="store_true", help="do not encode/write outputs (throughput runs)")
    ap.add_argument("--keep_staged", action="store_true",
                    help="--input_dir: also write the staged frame copies (the reference's work_dir/frames files); the "
                         "frames are staged in memory either way, with the same pixels")
    ap.add_argument("--png_writer", choices=["fast", "pil", "gpu"], default="pil",
                    help="PNG outputs: 'pil' (default) = Pillow's encoder at its defaults, byte-identical to the "
                         "reference's files; 'fast' = Up filter + zlib RLE deflate (pngio.py: ~6x faster than Pillow's "
                         "default encoder, files within a few percent of its size, opt-in); 'gpu' = the whole file "
                         "built on the GPU that styled the frame (csrc/png_enc.hip: Up filter, per-scanline dynamic "
                         "Huffman blocks, CRC and Adler-32 on the device), the host only writes bytes.  The pixels are "
                         "identical either way")
    ap.add_argument("--png_compress_level", type=int, default=None, choices=range(10), metavar="0-9",
                    help="Pillow's PNG encoder at this zlib level (overrides --png_writer); the pixels are the same "
                         "at every level, only the file size and the encode time change")
    return ap


def reject_out_of_scope(args) -> None:
    bad = []
    if args.model_type in ("magenta", "torch7"):
        bad.append(f"--model_type {args.model_type}")
    for s in SLOTS:
        if getattr(args, f"model_{s}") and (getattr(args, f"model_{s}_type") in ("magenta", "torch7")
                                             or str(getattr(args, f"model_{s}")).lower() in ("magenta",)
                                             or str(getattr(args, f"model_{s}")).endswith(".t7")):
            bad.append(f"--model_{s} (magenta/torch7)")
    if args.device != "cuda":
        bad.append(f"--device {args.device} (this engine runs on MI355X only; there is no CPU path)")
    if bad:
        _log("[error] not supported by the MI355X engine: " + ", ".join(bad))
        sys.exit(2)


# ----------------------------------------------------------------------------- host I/O helpers
# EXIF Orientation (tag 0x0112) -> counter-clockwise PIL rotation that uprights the image
_EXIF_UPRIGHT = {3: 180, 6: 270, 8: 90}


def _get_image_with_exif_pil(image_path: str):
    """EXIF-normalised RGB image (pipeline.py:171-187: orientations 3/6/8 rotated upright, others
    untouched; JPEG's legacy _getexif table, absent on other formats)."""
    from PIL import Image
    img = Image.open(image_path)
    tags = getattr(img, "_getexif", lambda: None)() or {}
    angle = _EXIF_UPRIGHT.get(tags.get(0x0112))
    if angle is not None:
        img = img.rotate(angle, expand=True)
    img.load()
    return img if img.mode == "RGB" else img.convert("RGB")  # (convert of an RGB image is a copy)


def sh(cmd: str, check=True):
    _log(f"$ {cmd}")
    r = subprocess.run(cmd, shell=True)
    if check and r.returncode != 0:
        _log(f"[sh][ERROR] exit {r.returncode}")
        sys.exit(r.returncode)
    return r.returncode


def _require_ffmpeg():
    if shutil.which("ffmpeg") is None:
        _log("[error] video mode needs ffmpeg on PATH (frame extract/assemble, pipeline.py:384-419, 2128-2150)")
        sys.exit(2)


def extract_frames(input_video: Path, frames_dir: Path, fps, scale, img_ext: str, jpeg_quality: int, canvas_wh=None):
    """pipeline.py:384-419 (ffmpeg subprocess)."""
    _require_ffmpeg()
    frames_dir.mkdir(parents=True, exist_ok=True)
    vf = []
    if canvas_wh:
        cw, ch = canvas_wh
        vf.append(f"scale={cw}:{ch}:flags=lanczos:force_original_aspect_ratio=decrease")
        vf.append(f"pad={cw}:{ch}:(ow-iw)/2:(oh-ih)/2:color=black")
    elif scale:
        vf.append(f"scale='if(gte(iw,ih),{scale},-2)':'if(gte(ih,iw),{scale},-2)':flags=lanczos")
    if fps:
        vf.append(f"fps={fps}")
    ext = "png" if img_ext.lower() == "png" else "jpg"
    pattern = frames_dir / f"frame_%04d.{ext}"
    vfs = f'-vf "{",".join(vf)}" ' if vf else ""
    sh(f'ffmpeg -y -i "{input_video}" {vfs}-c:v mjpeg -q:v {jpeg_quality} -pix_fmt yuvj420p "{pattern}"')


def assemble_video(frames_dir: Path, output_video: Path, in_fps, out_fps, prefix: str):
    """pipeline.py:2128-2150."""
    _require_ffmpeg()
    fr_in = f"-framerate {in_fps}" if in_fps else ""
    fr_out = f"-r {out_fps}" if out_fps else ""
    if sorted(frames_dir.glob(f"{prefix}_*.jpg")):
        pattern = frames_dir / f"{prefix}_%04d.jpg"
    elif sorted(frames_dir.glob(f"{prefix}_*.png")):
        pattern = frames_dir / f"{prefix}_%04d.png"
    else:
        _log("No styled frames found (jpg/png).")
        sys.exit(1)
    sh(f'ffmpeg -y {fr_in} -i "{pattern}" {fr_out} -c:v libx264 -pix_fmt yuv420p "{output_video}"')


def parse_blend_weights(weights_str: Optional[str], num_models: int) -> List[float]:
    """pipeline.py:502-511."""
    if not weights_str:
        return [1.0 / num_models] * num_models
    weights = [float(w) for w in weights_str.split(",")]
    if len(weights) != num_models:
        raise ValueError(f"Expected {num_models} weights, got {len(weights)}")
    if abs(sum(weights) - 1.0) > 1e-6:
        raise ValueError(f"Weights must sum to 1.0, got {sum(weights):.6f}")
    return weights


def parse_lab_weights(weights_str: Optional[str]):
    """pipeline.py:514-521."""
    if not weights_str:
        return 0.5, 0.5
    wL, wab = [float(w) for w in weights_str.split(",")]
    if abs(wL + wab - 1.0) > 1e-6:
        raise ValueError(f"LAB weights must sum to 1.0, got {wL + wab:.6f}")
    return wL, wab


def lab_weights_rest(weights_str: Optional[str], num_models: int) -> List[float]:
    """pipeline.py:1843-1852: weights of models B.. for the LAB blend (the reference's length rule)."""
    w = parse_blend_weights(weights_str, max(num_models - 1, 1))
    if len(w) == 1:
        return [1.0]
    if len(w) in (2, 3):
        return w
    return [1.0 / max(num_models - 1, 1)] * max(num_models - 1, 1)


def _pct_to_px(pct: float, H: int) -> int:
    """pipeline.py:278-282."""
    try:
        return int(round(max(0.0, float(pct)) * 0.01 * H))
    except Exception:
        return 0


def load_mask_fit(mask_path: str, target_hw, invert: bool, autofix: bool = True, force_transpose: bool = False) -> np.ndarray:
    """pipeline.py:284-353 without feathering: float32 HxW alpha in [0,1] (host file decode + NEAREST fit)."""
    return load_mask_u8(mask_path, target_hw, invert, autofix, force_transpose).astype(np.float32) / 255.0


def load_mask_u8(mask_path: str, target_hw, invert: bool, autofix: bool = True, force_transpose: bool = False) -> np.ndarray:
    """pipeline.py:292-347: the fitted (and optionally inverted) uint8 mask, before the feather."""
    from PIL import Image
    W_tgt, H_tgt = target_hw[1], target_hw[0]
    m_img = Image.open(mask_path).convert("L")
    mw, mh = m_img.size
    if force_transpose:
        m_img = m_img.transpose(Image.TRANSPOSE)
        mw, mh = m_img.size
    if autofix and (W_tgt != H_tgt):
        reason = None
        if (mw, mh) == (H_tgt, W_tgt):
            reason = "exact-dimension swap"
        else:
            def _dist(a, b):
                return abs(np.log(max(a, 1e-6)) - np.log(max(b, 1e-6)))
            ar_tgt, ar_mask, ar_sw = float(W_tgt) / float(H_tgt), float(mw) / float(mh), float(H_tgt) / float(W_tgt)
            if _dist(ar_mask, ar_sw) + 1e-6 < _dist(ar_mask, ar_tgt):
                reason = "aspect-ratio closer to swapped"
        if reason:
            _log(f"[mask][autofix] {Path(mask_path).name}: {reason}; applying Image.TRANSPOSE")
            m_img = m_img.transpose(Image.TRANSPOSE)
    m_img = m_img.resize((W_tgt, H_tgt), Image.Resampling.NEAREST)
    m = np.array(m_img, dtype=np.uint8)
    if invert:
        m = 255 - m
    return m


def _detect_transformer_type(checkpoint_path: str) -> str:
    """pipeline.py:72-79: NST_Train checkpoints have 'down1.' keys."""
    import torch
    state = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
    if isinstance(state, dict) and "state_dict" in state and isinstance(state["state_dict"], dict):
        state = state["state_dict"]
    return "nst" if any(k.startswith("down1.") for k in state.keys()) else "original"


def _load_checkpoint_compat(model, ckpt_path: str) -> None:
    """pipeline.py:554-569 (weights_only loads only: never unpickle arbitrary objects)."""
    import torch
    state = torch.load(ckpt_path, map_location="cpu", weights_only=True)
    if isinstance(state, dict) and "state_dict" in state and isinstance(state["state_dict"], dict):
        state = state["state_dict"]
    drop = ("running_mean", "running_var", "num_batches_tracked")
    state = {k: v for k, v in state.items() if not any(t in k for t in drop)}
    missing, unexpected = model.load_state_dict(state, strict=False)
    _log(f">> load_state_dict: missing={len(missing)} unexpected={len(unexpected)}")


def load_model(path: str, model_type: str, device, dtype: str, slot: str = "A", auto_nst: bool = True):
    """Model construction + load (pipeline.py:597-619; slots B..H always use the Johnson class for
    type transformer, :651-661 — kept)."""
    if model_type == "reconet":
        from .model import ReCoNet
        model, arch = ReCoNet(), "reconet"
    else:
        arch = _detect_transformer_type(path) if auto_nst else "original"
        if arch == "nst":
            from .transformer_net_nst import TransformerNet
            _log(f"[model] Detected NST_Train architecture for {path}")
        else:
            from .transformer_net import TransformerNet
        model = TransformerNet()
    _load_checkpoint_compat(model, path)
    model = model.to(device).eval()
    if dtype == "fp16m" and arch == "reconet":  # the split-precision head is built for the 128-channel nets
        _log("[backend] fp16m is built for the Johnson / NST nets; ReCoNet runs fp32s (the same +-1 LSB bar)")
        dtype = "fp32s"
    model.compute_dtype = dtype
    _log(f"[backend] {slot}: type={model_type} path={path} device={device} arch={arch} dtype={dtype}")
    return model, arch


# ----------------------------------------------------------------------------- the frame loop
class FrameSource:
    """Frames by index: files (PIL decode, optional --inference_res LANCZOS), --input_dir sources staged in memory
    (`staged`: (source path, JPEG quality or None) per frame), or a synthetic stream."""

    def __init__(self, files: Optional[List[Path]] = None, synthetic=None, infer_res: int = 0, staged=None):
        self.files = files if files is not None else ([s for s, _ in staged] if staged is not None else None)
        self.staged = staged
        self.synthetic = synthetic  # (n, h, w)
        self.infer_res = infer_res

    def __len__(self):
        return len(self.files) if self.files is not None else self.synthetic[0]

    def size(self, i: int):
        if self.files is None:
            return (self.synthetic[1], self.synthetic[2])
        from PIL import Image
        with Image.open(self.files[i]) as im:
            w, h = im.size
            if self.staged is not None:  # the staged copy is EXIF-upright: orientations 6 / 8 swap the sides
                try:
                    tags = getattr(im, "_getexif", lambda: None)() or {}
                except Exception:  # noqa: BLE001 -- unreadable EXIF: the raw copy is staged (_open_rgb)
                    tags = {}
                if _EXIF_UPRIGHT.get(tags.get(0x0112)) in (90, 270):
                    w, h = h, w
        return (h, w)

    def _open_rgb(self, i: int):
        from PIL import Image
        if self.staged is None:
            im = Image.open(self.files[i])
            im.load()
            return im if im.mode == "RGB" else im.convert("RGB")
        # the reference's --input_dir staging (pipeline.py:2577-2586): EXIF-upright RGB, re-saved as the staged
        # frame -- PNG (lossless: the decoded frame is that RGB image itself) or JPEG at --jpeg_quality, whose
        # encode -> decode round trip runs here in memory (the same bytes PIL writes, so the same pixels)
        src, q = self.staged[i]
        try:
            pil = _get_image_with_exif_pil(str(src))
        except Exception as e:  # noqa: BLE001 -- pipeline.py:2587-2589: the raw file is copied instead
            _log(f"[stage][WARN] EXIF-normalize failed for {src} ({e}); copying instead")
            im = Image.open(src)
            im.load()
            return im if im.mode == "RGB" else im.convert("RGB")
        if q is None:
            return pil
        # the round trip goes through an anonymous in-memory file with a real descriptor: Pillow encodes to a
        # descriptor with the GIL released (to a BytesIO it holds the GIL, so a thread pool would serialise)
        if not hasattr(os, "memfd_create"):  # (not Linux: same bytes through a BytesIO)
            import io
            buf = io.BytesIO()
            pil.save(buf, format="JPEG", quality=q)
            buf.seek(0)
            im = Image.open(buf)
            im.load()
            return im if im.mode == "RGB" else im.convert("RGB")
        with os.fdopen(os.memfd_create("nst_stage"), "w+b") as f:
            pil.save(f, format="JPEG", quality=q)
            f.seek(0)
            im = Image.open(f)
            im.load()
            return im if im.mode == "RGB" else im.convert("RGB")

    def load(self, i: int):
        """-> (original uint8 HxWx3, model-input uint8 hxwx3)."""
        if self.files is None:
            from .synthetic import make_frames
            f = make_frames(1, self.synthetic[1], self.synthetic[2], seed=10_000 + i)[0]
            return f, f
        from PIL import Image
        pil_rgb = self._open_rgb(i)
        pil_src = pil_rgb
        if self.infer_res > 0:  # pipeline.py:1089-1097
            w0, h0 = pil_rgb.size
            m0 = max(w0, h0)
            if m0 > self.infer_res:
                r = self.infer_res / float(m0)
                pil_src = pil_rgb.resize((int(round(w0 * r)), int(round(h0 * r))), Image.Resampling.LANCZOS)
        a = np.asarray(pil_rgb, dtype=np.uint8)
        return a, (a if pil_src is pil_rgb else np.asarray(pil_src, dtype=np.uint8))


def style_frames(args, frames_dir: Optional[Path], model_path, output_prefix: str, image_ext_out: str, device_str: str,
                 threads: int, stride: int, max_frames: Optional[int], smooth_lightness: bool, smooth_alpha: float,
                 jpeg_quality: int, io_preset: str, smooth_chroma: bool = False, chroma_alpha: float = 0.85,
                 blend: float = 1.0, image_mode: bool = False, save_map: Optional[Dict[int, str]] = None,
                 rank: int = 0, world: int = 1):
    """Same signature/behaviour as pipeline.py:527-2122 (in-scope paths), GPU-batched."""
    import torch
    from PIL import Image

    from .frames import plan_groups, rank0_share, run_pipeline
    t_setup = time.perf_counter()
    from .postproc import LabSmoother, blend_frames

    # one GPU per rank (several ranks may share a device with --dist_backend gloo: tests)
    dev = torch.device("cuda", rank % torch.cuda.device_count() if world > 1 else torch.cuda.current_device())
    torch.cuda.set_device(dev)
    blend = float(max(0.0, min(1.0, blend)))
    save_map = save_map or {}

    # ---- models: A + optional B..H (RGB blend, pipeline.py:1872-1879) ----
    slots, slot_letters = [], []
    model_a, arch_a = load_model(str(model_path), args.model_type, dev, args.dtype, "A")
    if arch_a == "nst" and io_preset in ("auto", "raw_255", "imagenet_255"):  # pipeline.py:610-614
        _log(f"[model] Auto-switching io_preset from '{io_preset}' to 'raw_01' for NST_Train model")
        io_preset = "raw_01"
    slots.append((model_a, io_preset))
    slot_letters.append(0)
    for li, s in enumerate(SLOTS, start=1):
        p = getattr(args, f"model_{s}", None)
        if not p:
            continue
        t = getattr(args, f"model_{s}_type", None) or args.model_type
        ip = getattr(args, f"io_preset_{s}", None) or io_preset
        m, _ = load_model(p, t, dev, args.dtype, s.upper(), auto_nst=False)
        slots.append((m, ip))
        slot_letters.append(li)
    # pipeline.py:1519-1520: the standard path blends only when one of B, C, D is in use, and counts models as
    # 1 + B + C + D (slots E..H join the outputs list but the weights cover the first num_models of it)
    n_blend = 1 + sum(1 for s in SLOTS[:3] if getattr(args, f"model_{s}", None))
    regions = None
    if args.region_mode and (args.region_optimize or n_blend > 1):
        from .regions import RegionCompositor
        regions = RegionCompositor(args, dev)
        _log(f"[region] mode={args.region_mode} optimize={regions.optimized} seed={regions.seed}")
    if n_blend > 1 and getattr(args, "blend_models_lab", False):
        # LAB blend (pipeline.py:1841-1870): L from A, a/b from the weighted mix of the others
        lab_wl, lab_wab = parse_lab_weights(getattr(args, "blend_models_lab_weights", None))
        lab_rest = lab_weights_rest(args.blend_models_weights, n_blend)
        weights = [lab_wl, lab_wab] + lab_rest
        _log(f"[blend] LAB blend: L={lab_wl},ab={lab_wab},rest={lab_rest}")
    else:
        weights = parse_blend_weights(args.blend_models_weights, n_blend) if n_blend > 1 else [1.0]
    _log(f"[cfg] io_preset={io_preset} models={len(slots)} weights={weights} dtype={args.dtype} gpus={world} batch={args.batch}")
    _log(f">> smoothing: {smooth_lightness}  alpha={smooth_alpha}  |  blend={blend}")

    # ---- frames ----
    if args.synthetic:
        m = re.match(r"^\s*(\d+)\s*[xX]\s*(\d+)\s*$", args.synthetic)
        if not m:
            _log(f"[error] --synthetic expects WxH, got {args.synthetic}")
            sys.exit(2)
        n_syn = int(args.synthetic_frames)
        if max_frames:
            n_syn = min(n_syn, int(max_frames))
        src = FrameSource(synthetic=(n_syn, int(m.group(2)), int(m.group(1))))
        names = [f"frame_{i + 1:04d}" for i in range(n_syn)]
    else:
        staged = getattr(args, "_staged_sources", None)
        if staged is not None:  # --input_dir: frame_{i:04d} staged in memory (prepare); only .png/.jpg/.jpeg
            # staged frames are styled (pipeline.py:1019-1021 filters frames_dir by suffix)
            entries = [(f"frame_{i:04d}", s) for i, s in enumerate(staged, start=1)
                       if Path(s[0]).suffix.lower() in {".png", ".jpg", ".jpeg"}]
        else:
            files = sorted(p for p in frames_dir.iterdir() if p.is_file() and p.name.startswith("frame_")
                           and p.suffix.lower() in {".png", ".jpg", ".jpeg"})
            entries = [(p.stem, p) for p in files]
        if stride and stride > 1:
            entries = entries[::stride]
        if max_frames:
            entries = entries[:max_frames]
        if not entries:
            _log(f"[error] No frames found to style in: {frames_dir}")
            sys.exit(1)
        ir = int(getattr(args, "inference_res", 0) or 0)
        src = (FrameSource(staged=[e[1] for e in entries], infer_res=ir) if staged is not None
               else FrameSource(files=[e[1] for e in entries], infer_res=ir))
        names = [e[0] for e in entries]
    _log(f"[debug] found {len(src)} staged frame(s)")

    if getattr(args, "mask_dir", None) and not getattr(args, "mask", None) and not args.synthetic:
        md = Path(args.mask_dir)
        missing = [nm for nm in names if not (md / f"mask_{nm.split('_')[-1]}.png").exists()]
        if missing and len(missing) == len(names):
            _log(f"[mask][ERROR] --mask_dir set to {md} but no masks like mask_0001.png were found.")
            sys.exit(2)
        if missing:
            _log(f"[mask][WARN] {len(missing)}/{len(names)} mask(s) missing under {md}.")

    pool = ThreadPoolExecutor(max_workers=max(1, threads))
    prof = _PipeProf()
    with prof("size_scan"):  # header reads (a PNG's EXIF lookup decodes it): on the pool
        sizes = list(pool.map(src.size, range(len(src))))
    # with --flow_ema rank 0 runs every frame's temporal stage (flow + fused EMA + LAB EMA + blend): a lighter share
    # of each group (frames.rank0_share).  Otherwise its ordered stage is the LAB EMA over 1-3 byte planes per
    # pixel (negligible), and every rank takes a full share.
    bsz = max(1, args.batch)
    flow_mode = bool(getattr(args, "flow_ema", False))
    r0 = rank0_share(world, bsz) if flow_mode else bsz
    caps = [r0] + [bsz] * (world - 1)
    groups = plan_groups(sizes, world, bsz, r0)
    need_orig = blend < 1.0 or bool(args.mask or args.mask_dir) or (flow_mode and bool(getattr(args, "motion_blend", False)))

    # host decode runs ahead of the GPU: this rank's next group(s) are loading on the pool while a group is
    # stylized (and the previous group's encodes drain), so decode, GPU step and encode overlap
    from .frames import shard
    my_shards = [shard(g, world, rank, caps) for g in groups]
    shard_pos = {tuple(sh): k for k, sh in enumerate(my_shards) if sh}
    loads = {}
    prefetch_depth = 2

    pinned = {}  # shard k -> page-locked [n, h, w, 3] the loaders decode into (one H2D copy per group, async)

    def _load_into(f, buf, j):
        a, b = src.load(f)
        np.copyto(buf[j], a)  # numpy releases the GIL for the copy
        return None if b is a else b

    def _submit(k):
        if 0 <= k < len(my_shards) and my_shards[k] and k not in pinned:
            sh = my_shards[k]
            h0, w0 = sizes[sh[0]]
            if all(sizes[f] == (h0, w0) for f in sh):
                buf = torch.empty((len(sh), h0, w0, 3), dtype=torch.uint8, pin_memory=True)
                pinned[k] = buf
                bn = buf.numpy()
                for j, f in enumerate(sh):
                    loads[f] = pool.submit(_load_into, f, bn, j)
            else:
                pinned[k] = None
                for f in sh:
                    if f not in loads:
                        loads[f] = pool.submit(src.load, f)

    # the reference fits model A's output to the content size; with --inference_res the model
    # input is smaller than the content
    def stylize(idx: List[int]):
        if not idx:
            h0, w0 = sizes[0]
            if flow_mode:
                return torch.empty((0, 15 * h0 * w0), dtype=torch.uint8, device=dev)
            return torch.empty((0, h0, w0, 6 if need_orig else 3), dtype=torch.uint8, device=dev)
        k = shard_pos.get(tuple(idx), -1)
        for j in range(k, k + 1 + prefetch_depth):
            _submit(j)
        buf = pinned.pop(k, None)
        with prof("wait_decode"):
            loaded = [(loads.pop(f) if f in loads else pool.submit(src.load, f)).result() for f in idx]
        with prof("h2d"):
            if buf is not None:  # decoded straight into page-locked memory; loaded = the model inputs if different
                orig = buf.to(dev, non_blocking=True)
                xin = orig if loaded[0] is None else torch.from_numpy(np.stack(loaded)).to(dev)
            else:
                orig = torch.from_numpy(np.stack([a for a, _ in loaded])).to(dev, non_blocking=True)
                xin = orig if loaded[0][1] is loaded[0][0] else torch.from_numpy(np.stack([b for _, b in loaded])).to(dev)
        h0, w0 = orig.shape[1], orig.shape[2]
        fids = [f + 1 for f in idx]  # the reference's 1-based frame index (animations, rotation)
        if flow_mode:  # the temporal stage needs out01 before the ToPILImage truncation (pipeline.py:1884-1943)
            out01 = _out01_f32(xin, orig, fids, h0, w0)
            n = out01.shape[0]
            return torch.cat([out01.view(torch.uint8).reshape(n, -1), orig.reshape(n, -1)], dim=1)
        if regions is not None and regions.optimized:  # crops of the full-resolution frame (pipeline.py:1309)
            styled = regions.optimized_frames(dict(zip(slot_letters, slots)), orig, fids)
        elif regions is not None:
            from .regions import Source, forward_raw
            raw = [Source(forward_raw(m, xin, pr), pr) for m, pr in slots]
            styled = regions.standard(raw, orig, fids, n_blend, (h0, w0))
        elif n_blend == 1 and xin.shape[1:3] == orig.shape[1:3]:
            styled = slots[0][0].stylize_frames(xin, slots[0][1])
        elif n_blend == 1:
            styled = _slot_u8(slots[0][0], slots[0][1], xin, h0, w0)
        elif getattr(args, "blend_models_lab", False):
            from .postproc import blend_models_lab
            outs = [_slot_u8(m, pr, xin, h0, w0) for m, pr in slots[:n_blend]]
            styled = blend_models_lab(outs, lab_rest, lab_wl, lab_wab)
        else:
            styled = _blend_slots(slots[:n_blend], weights, xin, h0, w0)
        return torch.cat([styled, orig], dim=3) if need_orig else styled

    def _out01_f32(xin, orig, fids, h0, w0):
        """out01 [n,3,h0,w0] float32: the frame's styled result before ToPILImage (model A / RGB blend / LAB
        blend / region composite), for the temporal stage."""
        from .regions import Source, composite, crop_input, forward_raw
        if regions is not None and regions.optimized:
            return regions.optimized_frames(dict(zip(slot_letters, slots)), orig, fids, out_f32=True)
        if regions is not None:
            raw = [Source(forward_raw(m, xin, pr), pr) for m, pr in slots]
            return regions.standard(raw, orig, fids, n_blend, (h0, w0), out_f32=True)
        if n_blend > 1 and getattr(args, "blend_models_lab", False):  # to_tensor of the LAB-blended image
            from .postproc import blend_models_lab
            outs = [_slot_u8(m, pr, xin, h0, w0) for m, pr in slots[:n_blend]]
            u8 = blend_models_lab(outs, lab_rest, lab_wl, lab_wab)
            return crop_input(u8, (0, 0, w0, h0), (h0, w0))
        # model A alone, or the RGB blend: zeros + w_i * out_i, clamp -- one all-ones region of the compositor
        raw = [Source(forward_raw(m, xin, pr), pr) for m, pr in slots[:n_blend]]
        ones = torch.ones((1, h0, w0), dtype=torch.float32, device=dev)
        return composite(raw, [[(i, w) for i, w in enumerate(weights[:n_blend])]], ones, None, out_f32=True)

    lab = LabSmoother(dev, smooth_lightness, smooth_alpha, smooth_chroma, chroma_alpha)
    flow = None
    if flow_mode:
        from .temporal import FlowSmoother
        flow = FlowSmoother(True, float(args.flow_alpha), max(1, int(args.flow_downscale or 1)), args.flow_method)
    mask_cache = {}
    pending = []
    t_start = time.perf_counter()
    done = [0]

    # Output stages (frames.run_pipeline).  The frame's owner stylizes it and, at the end, D2Hs and encodes it on its
    # own PCIe link and host pool; the only ordered work is the LAB EMA (pipeline.py:1942-1978), which rank 0 runs
    # over the planes it smooths (1 byte per pixel by default) -- or, with --flow_ema, the whole temporal chain over
    # [out01 | orig], returning finished frames.  Mask composite and blend (pipeline.py:1984-2092) run on the owner.
    ordered_lab = (lab.sl or lab.sc) and not flow_mode

    def stylize_send(idx: List[int]):
        full = stylize(idx)
        if flow_mode:
            return full, None
        if ordered_lab:
            return lab.planes(full[..., :3] if need_orig else full), full
        return None, full

    def root_post(g: List[int], full):
        h0, w0 = sizes[g[0]]
        if lab.hw is not None and lab.hw != (h0, w0):
            _log(f"[size][reset] frame dims changed {lab.hw} -> {(h0, w0)}; resetting EMA caches")
            lab.reset()
            if flow is not None:
                flow.reset()
        if not flow_mode:
            return lab.smooth_planes(full, (h0, w0)) if ordered_lab else None
        # unpack [out01 f32 | orig u8] and run the temporal stage in frame order
        from .temporal import motion_alpha, planar_to_u8
        nb = 3 * h0 * w0 * 4
        out01 = full[:, :nb].contiguous().view(torch.float32).reshape(len(g), 3, h0, w0)
        orig = full[:, nb:].contiguous().reshape(len(g), h0, w0, 3)
        # None for the first frame of a run (no previous frame); the batch's flows come in one call
        fused, flows = flow.batch(out01, orig)
        motion = None
        if getattr(args, "motion_blend", False):  # pipeline.py:2072-2080 alpha from this frame's flow
            motion = [None if fl is None else motion_alpha(fl, blend) for fl in flows]
        styled = lab(planar_to_u8(torch.stack(fused)))
        lab.hw = (h0, w0)
        if need_orig:
            styled_in = styled
            styled = blend_frames(styled, orig, blend, _masks_for(g, h0, w0), args.composite_mode)
            if motion is not None:  # frames with a flow and no mask: the motion-adaptive blend replaces it
                for j, f in enumerate(g):
                    if motion[j] is not None and not _has_mask(f):
                        styled[j:j + 1] = blend_frames(styled_in[j:j + 1], orig[j:j + 1], 1.0, motion[j][None], "keep")
        return styled

    def ret_spec(g: List[int]):
        h0, w0 = sizes[g[0]]
        if flow_mode:
            return (h0, w0, 3), torch.uint8
        return ((lab.nplanes, h0 * w0), torch.uint8) if ordered_lab else None

    def emit(idx: List[int], rows, full):
        if not idx:
            return
        if flow_mode:
            styled = rows
        else:
            styled = full[..., :3].contiguous() if need_orig else full
            if ordered_lab:
                styled = lab.merge(styled, rows)
            if need_orig:
                h0, w0 = styled.shape[1], styled.shape[2]
                styled = blend_frames(styled, full[..., 3:].contiguous(), blend, _masks_for(idx, h0, w0),
                                      args.composite_mode)
        gpu_png = (getattr(args, "png_writer", "pil") == "gpu" and not args.no_save
                   and getattr(args, "png_compress_level", None) is None and not any(_out_path(f)[1] for f in idx))
        with prof("d2h"):
            # page-locked D2H on a copy stream behind the frames' last kernel; the encoders wait for its event, so
            # this thread goes on queueing the next group's forward instead of waiting for the GPU.  --png_writer gpu:
            # the group's finished PNG files (and their sizes) instead of the pixels
            if gpu_png:
                from .pngio import encode_png_gpu
                src, sizes_d = encode_png_gpu(styled)
            else:
                src, sizes_d = styled, None
            host_t = torch.empty(src.shape, dtype=torch.uint8, pin_memory=True)
            host_sz = torch.empty(src.shape[0], dtype=torch.int64, pin_memory=True) if gpu_png else None
            copy_stream.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(copy_stream):
                host_t.copy_(src, non_blocking=True)
                if gpu_png:
                    host_sz.copy_(sizes_d, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(copy_stream)
            src.record_stream(copy_stream)
            if gpu_png:
                sizes_d.record_stream(copy_stream)
        # one waiter thread per run waits for the copy's event and then hands the frames to the encoder pool, so no
        # pool thread sits blocked on the GPU (the pool also decodes the next groups)
        pending.append(waiter.submit(_hand_off, ev, host_t, list(idx) if not args.no_save else [], host_sz))
        del host_t  # the waiter holds it until the copy is done; the savers' row views keep it alive after that
        _reap_pending()
        if not args.no_save:
            written.extend(idx)
        done[0] += len(idx)
        el = time.perf_counter() - t_start
        who = f" rank {rank}" if world > 1 else ""
        _log(f"[frame]{who} {done[0]}/{len(src) if world == 1 else sum(len(sh) for sh in my_shards)} styled  "
             f"({done[0] / max(el, 1e-9):.2f} frames/s)")

    def _has_mask(f):  # pipeline.py:1985-1993 mask_used: a --mask, or this frame's --mask_dir file exists
        if getattr(args, "mask", None):
            return True
        if not getattr(args, "mask_dir", None) or args.synthetic:
            return False
        return (Path(args.mask_dir) / f"mask_{names[f].split('_')[-1]}.png").exists()

    def _masks_for(g, h0, w0):
        mfile_global = getattr(args, "mask", None)
        if not mfile_global and not getattr(args, "mask_dir", None):
            return None
        ms = []
        any_mask = False
        for f in g:
            mfile = mfile_global
            if not mfile and not args.synthetic:
                cand = Path(args.mask_dir) / f"mask_{names[f].split('_')[-1]}.png"
                mfile = str(cand) if cand.exists() else None
            if mfile is None:
                # no mask for this frame -> no composite (pipeline.py:1985-1993): the alpha that
                # leaves S unchanged is 1 for 'keep' and 0 for 'replace'
                ident = 1.0 if args.composite_mode == "keep" else 0.0
                ms.append(torch.full((h0, w0), ident, dtype=torch.float32, device=dev))
                continue
            any_mask = True
            key = (mfile, h0, w0)
            if key not in mask_cache:
                # pipeline.py:2001-2003: feather radius from --mask_feather_pct of the target height,
                # at least --mask_feather; the Gaussian feather runs on the GPU (nst_mask_feather)
                fpx = _pct_to_px(getattr(args, "mask_feather_pct", 0.0) or 0.0, h0)
                if getattr(args, "mask_feather", 0) and args.mask_feather > 0:
                    fpx = max(fpx, int(args.mask_feather))
                m8 = load_mask_u8(mfile, (h0, w0), bool(args.mask_invert), bool(args.mask_autofix),
                                  bool(args.mask_force_transpose))
                if fpx > 0:
                    from .postproc import feather_masks
                    mask_cache[key] = feather_masks(torch.from_numpy(m8)[None].to(dev), fpx)[0]
                else:
                    mask_cache[key] = torch.from_numpy(m8.astype(np.float32) / 255.0).to(dev)
            ms.append(mask_cache[key])
        if not any_mask:
            return None
        return torch.stack(ms)

    copy_stream = torch.cuda.Stream(dev)
    waiter = ThreadPoolExecutor(max_workers=1)

    def _hand_off(ev, host_t, idx, host_sz=None):
        ev.synchronize()
        host = host_t.numpy()
        # each save holds a row view of the page-locked buffer (numpy keeps the tensor as the view's base), so the
        # buffer is released when the group's last save ends -- not held for the whole run
        if host_sz is not None:  # finished PNG files from the GPU: write their bytes
            sz = host_sz.tolist()
            return [pool.submit(_write_file, host[j, :sz[j]], f) for j, f in enumerate(idx)]
        return [pool.submit(_save, host[j], f) for j, f in enumerate(idx)]

    saves = []  # save futures of handed-off groups, reaped as they finish (errors surface at the next reap)

    def _reap_pending(final: bool = False):
        keep = []
        for p in pending:
            if final or p.done():
                saves.extend(p.result())
            else:
                keep.append(p)
        pending[:] = keep
        left = []
        for q in saves:
            if final or q.done():
                q.result()
            else:
                left.append(q)
        saves[:] = left

    def _out_path(f: int):
        """frame f's output file and whether it is a JPEG (pipeline.py:2099-2119)"""
        save_as_jpg = image_ext_out.lower() == "jpg"
        if image_mode and (f + 1) in save_map:
            out_path = Path(save_map[f + 1])
            save_as_jpg = out_path.suffix.lower() in (".jpg", ".jpeg")
        else:
            idx_str = names[f].split("_")[-1]
            base = frames_dir if frames_dir is not None else Path(args.work_dir)
            out_path = (base / f"{output_prefix}_{idx_str}").with_suffix(".jpg" if save_as_jpg else ".png")
        return out_path, save_as_jpg

    def _write_file(data: np.ndarray, f: int):
        out_path, _ = _out_path(f)
        out_path.parent.mkdir(parents=True, exist_ok=True)
        with open(out_path, "wb") as fh:
            fh.write(memoryview(data))
        return str(out_path)

    def _save(img: np.ndarray, f: int):
        out_img = Image.fromarray(img)
        out_path, save_as_jpg = _out_path(f)
        out_path.parent.mkdir(parents=True, exist_ok=True)
        if save_as_jpg:
            out_img.save(out_path, format="JPEG", quality=int(jpeg_quality))
        elif getattr(args, "png_compress_level", None) is not None:
            out_img.save(out_path, compress_level=int(args.png_compress_level))
        elif getattr(args, "png_writer", "pil") == "fast":  # same pixels as Pillow's file (pngio docstring)
            from .pngio import write_png
            write_png(out_path, img)
        else:
            out_img.save(out_path)
        return str(out_path)

    written: List[int] = []
    if ordered_lab or flow_mode:
        run_pipeline(groups, world, rank, stylize_send, root_post, emit, ret_spec, dev, caps)
    else:  # no ordered stage: every rank runs its frames start to finish, no exchange
        from .frames import agree_ok
        for sh in my_shards:  # one entry per group on every rank (empty where this rank has no frames of it)
            err = None
            if sh:
                try:
                    _, full = stylize_send(sh)
                    emit(sh, None, full)
                except Exception as e:  # noqa: BLE001 -- re-raised below, after the other ranks have heard of it
                    err = e
            if world > 1:  # keep the ranks in step on errors, as run_pipeline does (RankFailed on the healthy ones)
                agree_ok(err is None, dev)
            if err is not None:
                raise err
    with prof("drain_saves"):
        _reap_pending(final=True)
    waiter.shutdown()
    pool.shutdown()
    prof.report(rank)
    el = time.perf_counter() - t_start
    LAST_RUN_STATS.update(frames=len(src), seconds=el, setup_seconds=t_start - t_setup, rank=rank,
                          written=[names[f] for f in written])
    if os.environ.get("NST_PIPE_WRITTEN"):  # diagnostics: the frames this rank encoded and wrote (tests)
        import json
        with open(os.path.join(os.environ["NST_PIPE_WRITTEN"], f"rank{rank}.json"), "w") as fh:
            json.dump({"rank": rank, "world": world, "written": [names[f] for f in written], "loop_seconds": el,
                       "setup_seconds": t_start - t_setup}, fh)
    if rank == 0:
        _log(f"Styled {len(src)}/{len(src)} frames in {el:.2f}s ({len(src) / max(el, 1e-9):.2f} frames/s)")


class _PipeProf:
    """Wall time of the frame loop's host-side phases on the main thread (NST_PIPE_PROF=1 prints them)."""

    def __init__(self):
        self.on = os.environ.get("NST_PIPE_PROF", "0") == "1"
        self.t: Dict[str, float] = {}

    def __call__(self, name: str):
        import contextlib

        if not self.on:
            return contextlib.nullcontext()

        @contextlib.contextmanager
        def cm():
            t0 = time.perf_counter()
            try:
                yield
            finally:
                self.t[name] = self.t.get(name, 0.0) + time.perf_counter() - t0
        return cm()

    def report(self, rank: int):
        if self.on:
            _log(f"[pipe-prof rank {rank}] " + " ".join(f"{k}={v:.3f}s" for k, v in self.t.items()))


def _slot_u8(model, preset, xin, h0, w0):
    """One slot's frames as the reference's to_pil(out.clamp(0,1)): decoded, fitted to the content
    size (bilinear, pipeline.py:1512-1516), clamped, truncated to uint8."""
    import torch

    from . import _lib
    from ._lib import check, lib
    dev = xin.device
    eng = model.engine(dev)
    n, h, w, _ = xin.shape
    oh, ow = eng.output_hw(h, w)
    if (oh, ow) == (h, w) == (h0, w0):
        return model.stylize_frames(xin, preset)
    y = torch.empty((n, 3, oh, ow), dtype=torch.float32, device=dev)
    eng.forward_into(xin, _lib.NST_IO_U8_NHWC, n, h, w, _lib.PRESETS[preset], y, _lib.NST_IO_F32_NCHW)
    out = torch.empty((n, h0, w0, 3), dtype=torch.uint8, device=dev)
    check(lib().nst_decode_resize_u8(y.data_ptr(), n, oh, ow, _lib.PRESETS[preset], out.data_ptr(), h0, w0,
                                     _lib.stream_ptr(dev)), "nst_decode_resize_u8")
    return out


def _blend_slots(slots, weights, xin, h0, w0):
    """Raw f32 outputs of every slot -> nst_blend_models_u8 (decode, fit, weighted sum, clamp, truncation)."""
    import ctypes

    import torch

    from . import _lib
    from ._lib import check, lib
    dev = xin.device
    ys, presets = [], []
    for model, preset in slots:
        eng = model.engine(dev)
        n, h, w, _ = xin.shape
        oh, ow = eng.output_hw(h, w)
        y = torch.empty((n, 3, oh, ow), dtype=torch.float32, device=dev)
        eng.forward_into(xin, _lib.NST_IO_U8_NHWC, n, h, w, _lib.PRESETS[preset], y, _lib.NST_IO_F32_NCHW)
        ys.append(y)
        presets.append(_lib.PRESETS[preset])
    shapes = {tuple(y.shape) for y in ys}
    if len(shapes) != 1:
        raise _lib.NstError(f"model outputs differ in size {shapes}: the reference cannot blend them either")
    m = len(ys)
    out = torch.empty((xin.shape[0], h0, w0, 3), dtype=torch.uint8, device=dev)
    yp = (ctypes.c_void_p * m)(*[y.data_ptr() for y in ys])
    pr = (ctypes.c_int * m)(*presets)
    wt = (ctypes.c_float * m)(*[float(np.float32(w)) for w in weights])
    n, _, oh, ow = ys[0].shape
    check(lib().nst_blend_models_u8(yp, pr, wt, m, n, oh, ow, out.data_ptr(), h0, w0, _lib.stream_ptr(dev)),
          "nst_blend_models_u8")
    return out


# ----------------------------------------------------------------------------- main
def _parse_canvas(s):
    if not s:
        return None
    m = re.match(r"^\s*(\d+)\s*[xX]\s*(\d+)\s*$", str(s))
    if not m:
        _log(f"[canvas][ERROR] Expected WxH (e.g., 1920x1080), got: {s}")
        sys.exit(2)
    return int(m.group(1)), int(m.group(2))


def prepare(args):
    """Mode decision + staging (pipeline.py:2430-2606). Returns (frames_dir, model_path, save_map, image_mode, video_mode)."""
    canvas_wh = _parse_canvas(getattr(args, "canvas", None))
    for k in ("input_video", "output_video", "input_image", "output_image", "input_dir", "output_dir"):
        v = getattr(args, k, None)
        if v is not None and str(v).strip() == "":
            setattr(args, k, None)
    if getattr(args, "pattern", None) in (None, ""):
        args.pattern = f"*.{args.image_ext}"
    image_single = bool(args.input_image) and bool(args.output_image)
    image_batch = bool(args.input_dir) and bool(args.output_dir)
    video = bool(args.input_video) and bool(args.output_video)
    synthetic = bool(args.synthetic)
    if (image_single or image_batch) and video:
        _log("Provide exactly one of: (input_video & output_video) OR (input_image & output_image) OR (input_dir & output_dir).")
        sys.exit(2)
    if not (image_single or image_batch or video or synthetic):
        _log("Specify (input_video & output_video) OR (input_image & output_image) OR (input_dir & output_dir).")
        sys.exit(2)
    if not args.model:
        _log("[error] --model is required")
        sys.exit(2)
    model_path = Path(args.model).resolve()
    if model_path.suffix.lower() == ".t7":
        args.model_type = "torch7"
    if args.io_preset == "auto":
        args.io_preset = IO_PRESETS_AUTO.get(args.model_type, "imagenet_01")
        _log(f"[auto] io_preset resolved to '{args.io_preset}' for backend '{args.model_type}'")
    reject_out_of_scope(args)
    save_map: Dict[int, str] = {}
    base_work = Path(args.work_dir).resolve()
    if synthetic:
        return None, model_path, save_map, False, False
    work_dir = base_work / f"job_{uuid.uuid4().hex[:8]}" if (image_single or image_batch) else base_work
    frames_dir = work_dir / "frames"
    if frames_dir.exists() and video:
        shutil.rmtree(frames_dir, ignore_errors=True)
    frames_dir.mkdir(parents=True, exist_ok=True)
    if video:
        in_v = Path(args.input_video).resolve()
        if args.pre_fps:
            tmp = work_dir / f"prefps_{args.pre_fps}.mp4"
            _require_ffmpeg()
            sh(f'ffmpeg -y -i "{in_v}" -vf fps={args.pre_fps} -c:v libx264 -pix_fmt yuv420p "{tmp}"')
            in_v = tmp
        extract_frames(in_v, frames_dir, args.fps if not args.pre_fps else None, args.scale, args.image_ext,
                       args.jpeg_quality, canvas_wh)
    elif image_single:
        src = Path(args.input_image).resolve()
        ext = src.suffix.lower() if src.suffix.lower() in (".png", ".jpg", ".jpeg") else ".png"
        dst = frames_dir / f"frame_0001{ext}"
        pil = _get_image_with_exif_pil(str(src))
        if ext in (".jpg", ".jpeg"):
            pil.save(dst, format="JPEG", quality=max(1, min(95, int(args.jpeg_quality))))
        else:
            pil.save(dst)
        save_map[1] = str(Path(args.output_image).resolve())
    else:
        in_files = sorted(glob.glob(os.path.join(args.input_dir, args.pattern)))
        if not in_files:
            _log(f"No files matched: {args.input_dir}/{args.pattern}")
            sys.exit(2)
        Path(args.output_dir).mkdir(parents=True, exist_ok=True)

        # the reference's per-file staging copy (pipeline.py:2560-2590: EXIF-upright RGB re-saved as
        # frames/frame_{i:04d}{ext}, JPEG at --jpeg_quality) happens in memory when the frame is loaded
        # (FrameSource._open_rgb): a PNG copy decodes to that RGB image itself, a JPEG copy is re-encoded and
        # decoded from memory -- the same pixels without writing the staged files (--keep_staged writes them too)
        q = max(1, min(95, int(args.jpeg_quality)))
        args._staged_sources = [(Path(f).resolve(), q if Path(f).suffix.lower() in (".jpg", ".jpeg") else None)
                                for f in in_files]
        if getattr(args, "keep_staged", False):
            def stage(i_f):
                i, f = i_f
                src = Path(f).resolve()
                ext = src.suffix.lower()
                pil = _get_image_with_exif_pil(str(src))
                dst = frames_dir / f"frame_{i:04d}{ext}"
                if ext in (".jpg", ".jpeg"):
                    pil.save(dst, format="JPEG", quality=q)
                else:
                    pil.save(dst)
            with ThreadPoolExecutor(max_workers=max(1, int(getattr(args, "threads", 1) or 1))) as ex:
                list(ex.map(stage, enumerate(in_files, start=1)))
        for i, f in enumerate(in_files, start=1):
            src = Path(f).resolve()
            ext = src.suffix.lower()
            base = src.stem
            out_ext = ext if args.keep_ext else (".jpg" if args.image_ext.lower() == "jpg" else ".png")
            m = re.match(r"^frame_(\d+)$", base)
            out_stem = f"{args.output_prefix}_{m.group(1)}" if m else f"{base}{args.output_suffix or ''}"
            save_map[i] = str((Path(args.output_dir) / f"{out_stem}{out_ext}").resolve())
    return frames_dir, model_path, save_map, (image_single or image_batch), video


def _worker(rank: int, world: int, argv: List[str], port: int, prep, staged=None):
    import torch
    import torch.distributed as dist
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    args = build_parser().parse_args(argv)
    if staged is not None:  # --input_dir sources staged in memory by the parent's prepare()
        args._staged_sources = staged
    dev = torch.device("cuda", rank % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    if args.dist_backend == "nccl":  # RCCL over xGMI, one GPU per rank
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                                device_id=dev, timeout=timedelta(seconds=args.dist_timeout))
    else:  # gloo: frames travel through host memory (ranks may share a GPU)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                                timeout=timedelta(seconds=args.dist_timeout))
    try:
        frames_dir, model_path, save_map, image_mode, _ = prep
        _run_style(args, frames_dir, model_path, save_map, image_mode, rank, world)
    finally:
        dist.destroy_process_group()


def _run_style(args, frames_dir, model_path, save_map, image_mode, rank=0, world=1):
    return style_frames(args, frames_dir, model_path, output_prefix="styled_frame", image_ext_out=args.image_ext,
                        device_str=args.device, threads=args.threads, stride=args.stride, max_frames=args.max_frames,
                        smooth_lightness=args.smooth_lightness, smooth_alpha=args.smooth_alpha,
                        jpeg_quality=args.jpeg_quality, io_preset=args.io_preset, smooth_chroma=args.smooth_chroma,
                        chroma_alpha=args.chroma_alpha, blend=args.blend, image_mode=image_mode, save_map=save_map,
                        rank=rank, world=world)


def main(argv: Optional[List[str]] = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    args = build_parser().parse_args(argv)
    prep = prepare(args)
    frames_dir, model_path, save_map, image_mode, video = prep
    # re-parse inside workers with the resolved preset/model type
    resolved = argv + ["--io_preset", args.io_preset, "--model_type", args.model_type]
    if args.gpus > 1:
        import socket

        import torch.multiprocessing as mp
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        mp.start_processes(_worker, args=(args.gpus, resolved, port, prep, getattr(args, "_staged_sources", None)), nprocs=args.gpus, start_method="spawn")
    else:
        _run_style(args, frames_dir, model_path, save_map, image_mode)
    if video:
        in_fps = int(args.pre_fps) if args.pre_fps else (int(args.fps) if args.fps else None)
        out_fps = int(args.fps) if (args.pre_fps and args.fps) else None
        assemble_video(frames_dir, Path(args.output_video).resolve(), in_fps, out_fps, prefix="styled_frame")
        _log(f"\n Done. Styled video at: {Path(args.output_video).resolve()}")
    elif image_mode:
        written = sum(1 for v in save_map.values() if Path(v).exists())
        _log(f"Wrote {written}/{len(save_map)} image(s)")
    if args.clean_frames and frames_dir is not None:
        for pat in ("frame_*.png", "frame_*.jpg", "styled_frame_*.png", "styled_frame_*.jpg"):
            for p in frames_dir.glob(pat):
                p.unlink(missing_ok=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
