#!/usr/bin/env python3
"""run_videos.py — drop-in for the reference's env -> pipeline adapter (run_videos.py:1-296).

Same environment variables and slot mapping (MODEL_A..D, MODEL_*_TYPE, IO_PRESET[_A..D],
BLEND_WEIGHTS, SCALE, FPS, BLEND, SMOOTH_*, MAX_FRAMES, ...), building the same pipeline
command line (run_videos.py:144-274) for this package's pipeline, plus GPUS (frames
round-robin over N GPUs -> --gpus N), BATCH and DTYPE.  The pipeline runs as a subprocess,
as in the reference (run_videos.py:295).
"""
from __future__ import annotations

import os
import pathlib
import shlex
import subprocess
import sys
from typing import List, Optional


def getenv(name: str, default: Optional[str] = None) -> Optional[str]:
    v = os.getenv(name)
    return v if v is not None and v != "" else default


def getbool(name: str, default: bool = False) -> bool:
    v = os.getenv(name)
    if v is None:
        return default
    return v.lower() in {"1", "true", "yes", "on"}


def canonical_model_type(t: Optional[str]) -> str:
    t = (t or "").lower()
    return "transformer" if t == "pytorch" else t


def resolve_nonmagnet_model(path_or_name: str, model_type: str) -> str:
    """run_videos.py:51-65."""
    p = pathlib.Path(path_or_name)
    if p.is_absolute():
        return str(p)
    mt = canonical_model_type(model_type)
    if mt in {"pytorch", "transformer"}:
        return str(pathlib.Path(getenv("PYTORCH_DIR", "/app/models/pytorch"))
                   / (path_or_name if p.suffix else f"{path_or_name}.pth"))
    if mt == "torch7":
        return str(pathlib.Path(getenv("TORCH_DIR", "/app/models/torch")) / (path_or_name if p.suffix else f"{path_or_name}.t7"))
    if mt == "reconet":
        return str(pathlib.Path(getenv("TRANSFORMER_DIR", "/app/models/transformers")) / path_or_name)
    return str(p)


def add_slot(cmd: List[str], suffix: str, model_val, model_type, magenta_style, io_preset) -> None:
    """run_videos.py:115-141 (magenta slots are passed through; the pipeline rejects them)."""
    if not model_val:
        return
    mt = canonical_model_type(model_type) or "transformer"
    if mt == "magenta" or model_val.lower() == "magenta":
        cmd += [f"--model{suffix}", "magenta", f"--model{suffix}_type", "magenta"]
        if magenta_style:
            cmd += [f"--magenta_style{suffix}", magenta_style]
    else:
        cmd += [f"--model{suffix}", resolve_nonmagnet_model(model_val, mt)]
        cmd += ["--model_type" if suffix == "" else f"--model{suffix}_type", mt]
    if io_preset:
        cmd += ["--io_preset" if suffix == "" else f"--io_preset{suffix}", io_preset]


def build_pipeline_cmd(video_path: str) -> List[str]:
    """run_videos.py:144-274 for this package's pipeline."""
    out_dir = getenv("OUT_DIR", "/app/output")
    stem = pathlib.Path(video_path).stem
    output_video = str(pathlib.Path(out_dir) / f"{stem}{getenv('OUTPUT_SUFFIX', '')}.mp4")
    cmd = [sys.executable, "-m", "neuralstyletransferv1_amd.pipeline",
           "--input_video", video_path, "--output_video", output_video, "--output_dir", out_dir,
           "--scale", str(getenv("SCALE", "720")), "--fps", str(getenv("FPS", "24")),
           "--blend", str(getenv("BLEND", "0.9")),
           "--flow_method", getenv("FLOW_METHOD", "dis"), "--flow_downscale", str(getenv("FLOW_DOWNSCALE", "1"))]
    if getenv("PRE_FPS"):
        cmd += ["--pre_fps", getenv("PRE_FPS")]
    if getbool("SMOOTH_LIGHTNESS", False):
        cmd += ["--smooth_lightness"]
    if getenv("SMOOTH_ALPHA", "0.65") is not None:
        cmd += ["--smooth_alpha", str(getenv("SMOOTH_ALPHA", "0.65"))]
    if getbool("SMOOTH_CHROMA", False):
        cmd += ["--smooth_chroma"]
    if getenv("CHROMA_ALPHA"):
        cmd += ["--chroma_alpha", getenv("CHROMA_ALPHA")]
    if getbool("FLOW_EMA", False):
        cmd += ["--flow_ema", "--flow_alpha", str(getenv("FLOW_ALPHA", "0.7"))]
    for env, flag in (("MAX_FRAMES", "--max_frames"), ("STRIDE", "--stride"), ("JPEG_QUALITY", "--jpeg_quality"),
                      ("MAGENTA_TILE", "--magenta_tile"), ("MAGENTA_OVERLAP", "--magenta_overlap"),
                      ("MAGENTA_TARGET_RES", "--magenta_target_res"), ("MAGENTA_MODEL_ROOT", "--magenta_model_root"),
                      ("BLEND_WEIGHTS", "--blend_models_weights"), ("BLEND_MODELS_LAB_WEIGHTS", "--blend_models_lab_weights"),
                      ("DEVICE", "--device"), ("THREADS", "--threads"), ("IMAGE_EXT", "--image_ext"),
                      ("GPUS", "--gpus"), ("BATCH", "--batch"), ("DTYPE", "--dtype")):
        if getenv(env):
            cmd += [flag, str(getenv(env))]
    if getbool("CLEAN_FRAMES", False):
        cmd += ["--clean_frames"]
    if getbool("BLEND_MODELS_LAB", False):
        cmd += ["--blend_models_lab"]
    if getbool("MOTION_BLEND", False):
        cmd += ["--motion_blend"]
    if getenv("PIPELINE_ARGS"):
        cmd += shlex.split(getenv("PIPELINE_ARGS"))
    io_global = getenv("IO_PRESET")
    add_slot(cmd, "", getenv("MODEL_A"), getenv("MODEL_A_TYPE"), getenv("MAGENTA_STYLE"), getenv("IO_PRESET_A", io_global))
    for s in ("B", "C", "D"):
        add_slot(cmd, f"_{s.lower()}", getenv(f"MODEL_{s}"), getenv(f"MODEL_{s}_TYPE"), getenv(f"MAGENTA_STYLE_{s}"),
                 getenv(f"IO_PRESET_{s}"))
    return cmd


def main(argv: List[str]) -> int:
    if len(argv) < 2:
        print("usage: run_videos.py <video_path>")
        return 2
    cmd = build_pipeline_cmd(argv[1])
    print(f"[run] MAX_FRAMES={getenv('MAX_FRAMES') or ''}")
    print("[run]", " ".join(shlex.quote(x) for x in cmd))
    return subprocess.run(cmd).returncode


if __name__ == "__main__":
    sys.exit(main(sys.argv))
