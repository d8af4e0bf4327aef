"""The per-frame pipeline glue pinned to the REFERENCE's own pipeline.py.

tests/golden/pipeline_c0.npz holds outputs of /root/reference/pipeline.py run end to end in image mode on a 256x256
JPEG (configs[0]): every io_preset, LAB smoothing on / off / with chroma, blend 0.9, the reference's center_circle
mask in keep and replace+invert modes, and two 2-frame --input_dir EMA sequences (tests/golden/make_golden_pipeline.py,
which documents the torchvision / cv2 start-up shim it needs).

* CPU: the oracle's restatement of the chain (staging re-encode, preset, forward, decode, clamp, truncation, LAB EMA,
  mask, blend) reproduces every reference output bit-exactly -- so the oracle the other tests lean on is pinned to
  the reference's pipeline code, not only to its modules.
* GPU: the engine's CLI (pipeline.main, same arguments) against the same reference outputs, in the fp32 / fp32s /
  fp16m modes: the engine's pre-LAB frames within +-1 LSB of the reference's, the CLI's files exactly the reference's
  post chain applied to them (test_cli_vs_reference_pipeline's docstring).  With LAB smoothing a 1-LSB RGB difference
  before LittleCMS can move an L / a / b byte across a step, which LAB -> RGB turns into a few LSB, so the direct
  file comparison is bounded, not +-1.
"""
import io
import json
import os

import numpy as np
import pytest
import torch
from PIL import Image

from conftest import GOLDEN
from neuralstyletransferv1_amd import synthetic
from oracle import nst_oracle as O

Z = np.load(os.path.join(GOLDEN, "pipeline_c0.npz"))
META = json.loads(str(Z["meta"]))
INS = [os.path.join(GOLDEN, p) for p in META["inputs"]]
MASK = os.path.join(GOLDEN, META["mask"])
SD = synthetic.make_state_dict("johnson", 0)
# the presets whose decode range is not the default checkpoint's 0..255 raw output, each run by the reference with a
# checkpoint calibrated for it (make_golden_pipeline.py --calibrated: synthetic.make_state_dict(..., preset=...))
ZC = np.load(os.path.join(GOLDEN, "pipeline_c0_cal.npz"))
META_C = json.loads(str(ZC["meta"]))
CAL_PRESET = {c["name"]: c["ckpt_preset"] for c in META_C["cases"]["single"]}
_SD_CAL = {}


def _sd(name):
    """The checkpoint a case runs: the default one, or the preset-calibrated one of a *_cal case."""
    if name not in CAL_PRESET:
        return SD
    if name not in _SD_CAL:
        _SD_CAL[name] = synthetic.make_state_dict("johnson", 0, preset=CAL_PRESET[name])
    return _SD_CAL[name]


def _want(name, kind):
    if name in CAL_PRESET:
        return [ZC[f"out_{name}"]]
    return [Z[f"out_{name}"]] if kind == "single" else [Z[f"seq_{name}_{i}"] for i in range(len(INS))]


def _flag(args, name, default=None, cast=str):
    return cast(args[args.index(name) + 1]) if name in args else default


def _staged(path, q=85):
    """pipeline.py:2577-2586: EXIF-upright RGB re-saved as the staged JPEG at --jpeg_quality, then decoded"""
    buf = io.BytesIO()
    Image.open(path).convert("RGB").save(buf, format="JPEG", quality=q)
    buf.seek(0)
    return np.array(Image.open(buf).convert("RGB"))


def _oracle_chain(args, paths, sd=SD):
    preset = _flag(args, "--io_preset", "imagenet_255")
    preset = "imagenet_255" if preset == "auto" else preset  # pipeline.py:2518-2523 for transformer models
    ema = O.LabEMA("--no-smooth_lightness" not in args, _flag(args, "--smooth_alpha", 0.7, float),
                   "--smooth_chroma" in args, _flag(args, "--chroma_alpha", 0.85, float))
    blend = _flag(args, "--blend", 1.0, float)
    outs = []
    for p in paths:
        fr = _staged(p)
        u8 = ema(O.stylize_u8("johnson", sd, fr[None], preset)[0])
        alpha = None
        if "--mask" in args:
            alpha = O.load_mask_fit(MASK, fr.shape[:2], invert="--mask_invert" in args)
        outs.append(O.blend_u8(u8, fr, alpha, _flag(args, "--composite_mode", "keep"), blend))
    return outs


def _cases():
    out = [(c["name"], c["args"], "single") for c in META["cases"]["single"]]
    out += [(c["name"], c["args"], "single") for c in META_C["cases"]["single"]]
    return out + [(c["name"], c["args"], "seq") for c in META["cases"]["seq"]]


@pytest.mark.parametrize("name,args,kind", _cases(), ids=[c[0] for c in _cases()])
def test_oracle_reproduces_reference_pipeline(name, args, kind):
    """The oracle's chain == the reference pipeline.py's files, bit for bit."""
    torch.set_num_threads(4)
    got = _oracle_chain(args, INS[:1] if kind == "single" else INS, _sd(name))
    want = _want(name, kind)
    for g, w in zip(got, want):
        d = np.abs(g.astype(int) - w.astype(int))
        assert d.max() == 0, f"{name}: max |d| {d.max()} on {(d > 0).mean():.4%} of values"


def _cli_outputs(tmp_path, name, args, kind, dtype):
    from neuralstyletransferv1_amd import pipeline as P
    ck = tmp_path / f"johnson_0_{CAL_PRESET.get(name, 'default')}.pth"
    if not ck.exists():
        torch.save(_sd(name), ck)
    extra = [MASK if a == "MASK" else a for a in args]
    if kind == "single":
        out = tmp_path / f"{name}_{dtype}.png"
        argv = ["--input_image", INS[0], "--output_image", str(out), "--model", str(ck), "--dtype", dtype,
                "--work_dir", str(tmp_path / f"w_{name}_{dtype}")] + extra
        assert P.main(argv) == 0
        return [np.array(Image.open(out).convert("RGB"))], _want(name, kind)
    d_in, d_out = tmp_path / f"in_{name}_{dtype}", tmp_path / f"out_{name}_{dtype}"
    d_in.mkdir()
    for i, p in enumerate(INS):
        (d_in / f"frame_{i + 1:04d}.jpg").write_bytes(open(p, "rb").read())
    argv = ["--input_dir", str(d_in), "--output_dir", str(d_out), "--pattern", "*.jpg", "--model", str(ck),
            "--dtype", dtype, "--work_dir", str(tmp_path / f"w_{name}_{dtype}")] + extra
    assert P.main(argv) == 0
    got = [np.array(Image.open(d_out / f"styled_frame_{i + 1:04d}.png").convert("RGB")) for i in range(len(INS))]
    return got, [Z[f"seq_{name}_{i}"] for i in range(len(INS))]


# the file-level bound with lightness smoothing on: a 1-LSB pre-LAB difference moved across a LittleCMS L step comes
# back from LAB -> RGB as several LSB (the fraction bars carry the statistics).  Measured over these fixtures
# (gpurun_out/gpu_tests_r06_e.log): max 9 LSB for fp32 / fp32s, 11 for fp16m, every pre-LAB value within +-1
LAB_MAX_LSB = 12


def _post_chain(args, frames, pre):
    """The reference chain after the first ToPILImage (LAB EMA, mask, blend), restated by the oracle, applied to
    given pre-LAB frames."""
    ema = O.LabEMA("--no-smooth_lightness" not in args, _flag(args, "--smooth_alpha", 0.7, float),
                   "--smooth_chroma" in args, _flag(args, "--chroma_alpha", 0.85, float))
    blend = _flag(args, "--blend", 1.0, float)
    outs = []
    for fr, u8 in zip(frames, pre):
        alpha = None
        if "--mask" in args:
            alpha = O.load_mask_fit(MASK, fr.shape[:2], invert="--mask_invert" in args)
        outs.append(O.blend_u8(ema(u8), fr, alpha, _flag(args, "--composite_mode", "keep"), blend))
    return outs


def _cli_params():
    out = []
    for name, args, kind in _cases():
        preset = _flag(args, "--io_preset", "imagenet_255")
        for dtype in ("fp32", "fp32s", "fp16m"):
            if dtype == "fp16m" and name not in CAL_PRESET and preset in ("imagenet_01", "tanh", "raw_01"):
                continue  # the calibrated *_cal case of this preset runs it (docstring)
            out.append(pytest.param(name, args, kind, dtype, id=f"{name}-{dtype}"))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("name,args,kind,dtype", _cli_params())
def test_cli_vs_reference_pipeline(tmp_path, name, args, kind, dtype):
    """The engine CLI against the reference pipeline.py's files.  Decomposed so the bar is the north_star's +-1 LSB
    where the arithmetic differs and exact everywhere else: (1) the engine's pre-LAB frames of the staged input are
    within +-1 LSB of the reference's (the oracle's, which test_oracle_reproduces_reference_pipeline pins bit-exactly
    to the reference's outputs); (2) the CLI's files are EXACTLY the reference's post chain (LAB EMA, mask, blend)
    applied to those engine frames; (3) the files against the reference's files: without LAB every value within
    +-1 LSB; with LAB, which amplifies a pre-LAB 1-LSB difference to several LSB where a LittleCMS byte crosses a
    step, reported, with fp32 / fp32s <= 1 LSB on >= 99.9 % of values and fp16m (5-6 % of pre-LAB values off by
    one) <= 2 LSB on >= 98 %, and a max bound on every case.

    fp16m runs the imagenet_01 / tanh / raw_01 presets only with their calibrated checkpoints (the *_cal cases):
    the default synthetic checkpoint's raw output spans 0..255, which these presets decode at 1/58 .. 1/255 of the
    scale into mostly saturated frames, magnifying the 16-bit trunk's rounding 58-255x against an output LSB -- a
    checkpoint trained with such a preset outputs in its range, which is what *_cal stands for.
    fp32 / fp32s run every case."""
    preset = _flag(args, "--io_preset", "imagenet_255")
    preset = "imagenet_255" if preset == "auto" else preset
    sd = _sd(name)
    got, want = _cli_outputs(tmp_path, name, args, kind, dtype)
    paths = INS[:1] if kind == "single" else INS
    frames = [_staged(p) for p in paths]
    m = synthetic.build_module("johnson")
    m.load_state_dict(sd)
    m = m.to("cuda").eval()
    m.compute_dtype = dtype
    pre = m.stylize_frames(torch.from_numpy(np.stack(frames)).cuda(), preset).cpu().numpy()
    ref_pre = O.stylize_u8("johnson", sd, np.stack(frames), preset)
    dp = np.abs(pre.astype(int) - ref_pre.astype(int))
    assert dp.max() <= 1, f"pre-LAB max |d| {dp.max()}"
    exp = _post_chain(args, frames, list(pre))
    lab = "--no-smooth_lightness" not in args or "--smooth_chroma" in args
    for g, e, w in zip(got, exp, want):
        assert np.array_equal(g, e), f"CLI output differs from the reference post chain of its own pre-LAB frames"
        d = np.abs(g.astype(int) - w.astype(int))
        print(f"{name} {dtype}: pre-LAB max {dp.max()} ({(dp > 0).mean():.4%} off by one); vs reference file max |d| "
              f"{d.max()} LSB, values > 1 LSB {(d > 1).mean():.4%}")
        # the max bound holds where only the lightness is smoothed; with chroma smoothing a 1-LSB pre-LAB difference
        # near a gamut edge can come back from LittleCMS LAB -> RGB as a large jump on single pixels (133 LSB on one
        # value of ema_blend in fp16m, gpurun_out/gpu_tests_r06_f.log), which the exact decomposition above already
        # attributes to the reference's own post chain
        chroma = "--smooth_chroma" in args
        if not lab:
            assert d.max() <= 1
        elif dtype == "fp16m":
            assert (d > 2).mean() <= 2e-2 and (chroma or d.max() <= LAB_MAX_LSB), (d.max(), (d > 2).mean())
        else:
            assert (d > 1).mean() <= 1e-3 and (chroma or d.max() <= LAB_MAX_LSB), (d.max(), (d > 1).mean())
