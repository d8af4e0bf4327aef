"""End-to-end CLI runs on the GPU (image, batch-dir + mask + blend + multi-model, synthetic stream)
compared with the oracle's restatement of the same per-frame chain."""
import os

import numpy as np
import pytest
import torch
from PIL import Image

from conftest import GOLDEN
from neuralstyletransferv1_amd import pipeline as P
from neuralstyletransferv1_amd import synthetic
from oracle import nst_oracle as O

pytestmark = pytest.mark.gpu


def _ckpt(tmp_path, arch, seed):
    sd = synthetic.make_state_dict(arch, seed)
    p = tmp_path / f"{arch}_{seed}.pth"
    torch.save(sd, p)
    return str(p), sd


def _oracle_chain(arch_sds, weights, frames, preset, smooth=True, alpha=0.7, blend=1.0, masks=None, mode="keep"):
    """pipeline.py per-frame chain restated: models (+RGB blend) -> ToPILImage -> LAB EMA -> mask -> blend."""
    outs = []
    ema = O.LabEMA(smooth, alpha)
    for i, fr in enumerate(frames):
        x01 = O.to_tensor01(fr[None])
        acc = None
        for (arch, sd), w in zip(arch_sds, weights):
            with torch.no_grad():
                y = O.FORWARDS[arch](sd, O.encode(x01, preset))
                o = O.fit_to_content(O.decode(y, preset), fr.shape[0], fr.shape[1])
            acc = torch.zeros_like(o) if acc is None else acc
            acc += w * o
        out01 = acc.clamp(0, 1)
        u8 = O.to_pil_u8(out01)[0]
        u8 = ema(u8)
        m = None if masks is None else masks[i][..., None]
        outs.append(O.blend_u8(u8, fr, m, mode, blend))
    return outs


# After the LAB round trip (Pillow/LittleCMS, pipeline.py:1942-1978) a 1-LSB RGB difference before it can
# move an L / a / b byte across a quantisation step, which LAB -> RGB turns into a few LSB.  The engine's LAB
# stage is bit-exact (tests/test_gpu_parity.py), and test_pre_lab_within_1lsb_and_lab_attribution shows
# that every post-LAB difference is the round trip of a <= 1 LSB pre-LAB one; this bounds the result.
LAB_MAX_LSB = 8


def _close(a, b, max_lsb, frac=0.005):
    """every value within max_lsb, and at most frac of them more than 2 LSB apart"""
    d = np.abs(a.astype(int) - b.astype(int))
    print(f"max |d| {d.max()} LSB, > 1 LSB {(d > 1).mean():.4%}, > 2 LSB {(d > 2).mean():.4%}")
    assert (d > 2).mean() <= frac, f"{(d > 2).mean():.4%} of values differ by >2 LSB (max {d.max()})"
    assert d.max() <= max_lsb, f"max |d| {d.max()} > {max_lsb} LSB"


def test_single_image_cli_fp32(tmp_path):
    ck, sd = _ckpt(tmp_path, "johnson", 0)
    fr = synthetic.make_frames(1, 72, 96, seed=21)[0]
    inp, outp = tmp_path / "in.png", tmp_path / "out.png"
    Image.fromarray(fr).save(inp)
    rc = P.main(["--input_image", str(inp), "--output_image", str(outp), "--model", ck, "--io_preset", "raw_255",
                 "--work_dir", str(tmp_path / "w")])
    assert rc == 0
    got = np.array(Image.open(outp))
    ref = _oracle_chain([("johnson", sd)], [1.0], [fr], "raw_255")[0]
    _close(got, ref, LAB_MAX_LSB)


@pytest.mark.parametrize("preset,seed", [("raw_255", 0), ("imagenet_255", 1)])
def test_pre_lab_within_1lsb_and_lab_attribution(tmp_path, preset, seed):
    """fp32 CLI: (1) with --no-smooth_lightness the output (the stylised frame before the LAB stage) is
    within +-1 LSB of the oracle everywhere; (2) with LAB smoothing on, the output is exactly the
    reference's LAB EMA (Pillow/LittleCMS, oracle) applied to that GPU pre-LAB frame — so any larger
    difference from the oracle chain is the LAB round trip of a <= 1 LSB pre-LAB difference."""
    ck, sd = _ckpt(tmp_path, "johnson", seed)
    frames = synthetic.make_frames(2, 96, 128, seed=60 + seed)
    d_in = tmp_path / "in"
    d_in.mkdir()
    for i, f in enumerate(frames):
        Image.fromarray(f).save(d_in / f"frame_{i + 1:04d}.png")
    outs = {}
    for tag, extra in (("pre", ["--no-smooth_lightness"]), ("lab", ["--smooth_alpha", "0.65"])):
        d_out = tmp_path / f"out_{tag}"
        assert P.main(["--input_dir", str(d_in), "--output_dir", str(d_out), "--model", ck, "--io_preset", preset,
                       "--batch", "2", "--work_dir", str(tmp_path / f"w_{tag}")] + extra) == 0
        outs[tag] = [np.array(Image.open(d_out / f"styled_frame_{i + 1:04d}.png")) for i in range(2)]
    ref_pre = _oracle_chain([("johnson", sd)], [1.0], list(frames), preset, smooth=False)
    ref_lab = _oracle_chain([("johnson", sd)], [1.0], list(frames), preset, alpha=0.65)
    ema = O.LabEMA(True, 0.65)
    for i in range(2):
        d = np.abs(outs["pre"][i].astype(int) - ref_pre[i].astype(int))
        assert d.max() <= 1, f"pre-LAB max |d| {d.max()}"
        assert np.array_equal(outs["lab"][i], ema(outs["pre"][i])), "post-LAB output is not LAB(pre-LAB)"
        dl = np.abs(outs["lab"][i].astype(int) - ref_lab[i].astype(int))
        print(f"{preset} frame {i}: pre-LAB max {d.max()} ({(d > 0).mean():.4%} off), post-LAB max {dl.max()} "
              f"({(dl > 1).mean():.4%} > 1 LSB)")
        assert dl.max() <= LAB_MAX_LSB


def test_batch_dir_mask_blend_multimodel_fp32(tmp_path):
    ck_a, sd_a = _ckpt(tmp_path, "johnson", 0)
    ck_b, sd_b = _ckpt(tmp_path, "johnson", 5)
    frames = synthetic.make_frames(3, 64, 80, seed=30)
    d_in, d_out = tmp_path / "in", tmp_path / "out"
    d_in.mkdir()
    for i, f in enumerate(frames):
        Image.fromarray(f).save(d_in / f"frame_{i + 1:04d}.png")
    mask = os.path.join(GOLDEN, "masks", "center_circle.png")
    rc = P.main(["--input_dir", str(d_in), "--output_dir", str(d_out), "--model", ck_a, "--model_b", ck_b,
                 "--blend_models_weights", "0.6,0.4", "--io_preset", "imagenet_255", "--mask", mask, "--blend", "0.9",
                 "--smooth_alpha", "0.65", "--batch", "2", "--work_dir", str(tmp_path / "w")])
    assert rc == 0
    alpha = P.load_mask_fit(mask, (64, 80), False)
    ref = _oracle_chain([("johnson", sd_a), ("johnson", sd_b)], [0.6, 0.4], list(frames), "imagenet_255",
                        alpha=0.65, blend=0.9, masks=[alpha] * 3)
    for i in range(3):
        got = np.array(Image.open(d_out / f"styled_frame_{i + 1:04d}.png"))
        _close(got, ref[i], LAB_MAX_LSB)


def test_synthetic_stream_bf16_nst_and_reconet(tmp_path):
    for arch, model_type in (("nst", "transformer"), ("reconet", "reconet")):
        ck, _ = _ckpt(tmp_path, arch, 1)
        rc = P.main(["--synthetic", "160x96", "--synthetic_frames", "5", "--model", ck, "--model_type", model_type,
                     "--dtype", "bf16", "--batch", "2", "--work_dir", str(tmp_path / f"w_{arch}")])
        assert rc == 0
        outs = sorted((tmp_path / f"w_{arch}").glob("styled_frame_*.png"))
        assert len(outs) == 5
        assert np.array(Image.open(outs[0])).shape == (96, 160, 3)


def test_lab_blend_bit_exact_vs_oracle():
    """nst_blend_models_lab_u8 == pipeline.py:1854-1869 on Pillow/LittleCMS (2..4 models, zip rule)."""
    from neuralstyletransferv1_amd.postproc import blend_models_lab
    rng = np.random.default_rng(5)
    fr = [rng.integers(0, 256, (2, 33, 47, 3), dtype=np.uint8) for _ in range(4)]
    for m, rest, wl, wab in ((2, [1.0], 0.5, 0.5), (3, [0.25, 0.75], 0.3, 0.7), (4, [0.2, 0.3, 0.5], 0.5, 0.5),
                             (4, [0.6, 0.4], 0.9, 0.1)):
        dev = [torch.from_numpy(f).cuda() for f in fr[:m]]
        out = blend_models_lab(dev, rest, wl, wab).cpu().numpy()
        for i in range(2):
            ref = O.lab_blend_u8([f[i] for f in fr[:m]], rest, wl, wab)
            assert np.array_equal(out[i], ref), (m, rest, wl, wab, i)


def test_mask_feather_vs_restatement():
    """nst_mask_feather against the numpy restatement of cv2.GaussianBlur (parity unpinned: cv2 is
    absent; tolerance 1 LSB of the uint8 blur for float32 vs float64 taps)."""
    from neuralstyletransferv1_amd.postproc import feather_masks
    m = np.zeros((2, 61, 90), np.uint8)
    m[0, 10:40, 20:70] = 255
    m[1] = np.random.default_rng(2).integers(0, 256, (61, 90), dtype=np.uint8)
    for fpx in (1, 4, 13, 40):
        a = feather_masks(torch.from_numpy(m).cuda(), fpx).cpu().numpy()
        for i in range(2):
            ref = O.feather_mask_u8(m[i], fpx).astype(np.float32) / 255.0
            assert np.abs(a[i] - ref).max() <= 1.0 / 255.0 + 1e-7, (fpx, i)
            assert (np.abs(a[i] - ref) > 1e-7).mean() < 0.01


def test_cli_lab_blend_and_feathered_mask(tmp_path):
    """--blend_models_lab with three models and a feathered mask composite through the CLI."""
    cka, sda = _ckpt(tmp_path, "johnson", 0)
    ckb, sdb = _ckpt(tmp_path, "johnson", 1)
    ckc, sdc = _ckpt(tmp_path, "johnson", 2)
    frames = synthetic.make_frames(2, 48, 64, seed=8)
    d = tmp_path / "frames"
    d.mkdir()
    for i, f in enumerate(frames):
        Image.fromarray(f).save(d / f"frame_{i + 1:04d}.png")
    mask = np.zeros((48, 64), np.uint8)
    mask[8:40, 16:48] = 255
    Image.fromarray(mask).save(tmp_path / "mask.png")
    out_d = tmp_path / "out"
    rc = P.main(["--input_dir", str(d), "--output_dir", str(out_d), "--model", cka, "--model_b", ckb, "--model_c", ckc,
                 "--io_preset", "raw_255", "--blend_models_lab", "--blend_models_lab_weights", "0.4,0.6",
                 "--blend_models_weights", "0.5,0.5", "--mask", str(tmp_path / "mask.png"), "--mask_feather", "6",
                 "--no-smooth_lightness", "--work_dir", str(tmp_path / "w")])
    assert rc == 0
    alpha = O.feather_mask_u8(mask, 6).astype(np.float32) / 255.0
    outs = sorted(out_d.iterdir())
    assert len(outs) == 2
    for i, fr in enumerate(frames):
        per = []
        for sd in (sda, sdb, sdc):
            per.append(O.stylize_u8("johnson", sd, fr[None], "raw_255")[0])
        lab = O.lab_blend_u8(per, [0.5, 0.5], 0.4, 0.6)
        ref = O.blend_u8(lab, fr, alpha[..., None], "keep", 1.0)
        got = np.array(Image.open(outs[i]))
        _close(got, ref, LAB_MAX_LSB, frac=0.01)


def _lsb_report(got, ref):
    d = np.abs(got.astype(int) - ref.astype(int))
    return d, float((d <= 2).mean()), int(d.max())


def test_1080p_mask_blend_cli_vs_oracle(tmp_path):
    """configs[4] without DeepLab: 1080p frames, a per-frame mask directory (mask_####.png, the
    sky_swap.py output layout), --composite_mode keep, --blend 0.9, LAB smoothing 0.65 (run_videos.py
    defaults) through the CLI, fp32 parity mode against the oracle chain: u8 values within 2 LSB on
    >= 99.99 % of them; and the bf16 throughput mode (the bench kernels) at SSIM >= 0.98."""
    ck, sd = _ckpt(tmp_path, "johnson", 0)
    frames = synthetic.make_frames(2, 1080, 1920, seed=77)
    d_in, d_m = tmp_path / "in", tmp_path / "masks"
    d_in.mkdir()
    d_m.mkdir()
    src_mask = Image.open(os.path.join(GOLDEN, "masks", "center_circle.png")).convert("L")
    for i, f in enumerate(frames):
        Image.fromarray(f).save(d_in / f"frame_{i + 1:04d}.png")
        src_mask.rotate(15 * i).save(d_m / f"mask_{i + 1:04d}.png")
    masks = [P.load_mask_fit(str(d_m / f"mask_{i + 1:04d}.png"), (1080, 1920), False) for i in range(2)]
    ref = _oracle_chain([("johnson", sd)], [1.0], list(frames), "imagenet_255", alpha=0.65, blend=0.9,
                        masks=masks, mode="keep")
    for dtype in ("fp32", "bf16"):
        d_out = tmp_path / f"out_{dtype}"
        rc = P.main(["--input_dir", str(d_in), "--output_dir", str(d_out), "--model", ck, "--io_preset", "imagenet_255",
                     "--mask_dir", str(d_m), "--composite_mode", "keep", "--blend", "0.9", "--smooth_alpha", "0.65",
                     "--dtype", dtype, "--batch", "2", "--work_dir", str(tmp_path / f"w_{dtype}")])
        assert rc == 0
        for i in range(2):
            got = np.array(Image.open(d_out / f"styled_frame_{i + 1:04d}.png"))
            d, within2, dmax = _lsb_report(got, ref[i])
            print(dtype, i, "within 2 LSB", within2, "max", dmax, "ssim", O.ssim(got, ref[i]))
            if dtype == "fp32":
                assert within2 >= 0.9999 and dmax <= LAB_MAX_LSB, (within2, dmax)
            else:
                assert O.ssim(got, ref[i]) >= 0.98


def test_single_256_jpeg_cli_config0(tmp_path):
    """configs[0]: one 256x256 JPEG through the Johnson TransformerNet via the single-image CLI
    (io_preset auto -> imagenet_255 for transformer models, LAB smoothing on by default)."""
    ck, sd = _ckpt(tmp_path, "johnson", 3)
    fr = synthetic.make_frames(1, 256, 256, seed=256)[0]
    inp, outp = tmp_path / "in.jpg", tmp_path / "out.png"
    Image.fromarray(fr).save(inp, format="JPEG", quality=95)
    # the CLI stages the image EXIF-normalised and re-saved at --jpeg_quality (85), pipeline.py:2552-2561
    import io
    buf = io.BytesIO()
    Image.open(inp).convert("RGB").save(buf, format="JPEG", quality=85)
    decoded = np.array(Image.open(io.BytesIO(buf.getvalue())).convert("RGB"))
    rc = P.main(["--input_image", str(inp), "--output_image", str(outp), "--model", ck, "--model_type", "transformer",
                 "--work_dir", str(tmp_path / "w")])
    assert rc == 0
    got = np.array(Image.open(outp))
    ref = _oracle_chain([("johnson", sd)], [1.0], [decoded], "imagenet_255")[0]
    d, within2, dmax = _lsb_report(got, ref)
    assert got.shape == (256, 256, 3) and within2 >= 0.9999, (within2, dmax)


def test_inference_res_lanczos_cli(tmp_path):
    """--inference_res (pipeline.py:1089-1097): frames whose long side exceeds it are LANCZOS-downscaled
    for the model, the output is fitted back to the content size (pipeline.py:1512-1516, bilinear)."""
    ck, sd = _ckpt(tmp_path, "johnson", 4)
    fr = synthetic.make_frames(1, 120, 162, seed=31)[0]
    inp, outp = tmp_path / "in.png", tmp_path / "out.png"
    Image.fromarray(fr).save(inp)
    rc = P.main(["--input_image", str(inp), "--output_image", str(outp), "--model", ck, "--io_preset", "raw_255",
                 "--inference_res", "100", "--work_dir", str(tmp_path / "w")])
    assert rc == 0
    pil = Image.fromarray(fr)
    r = 100 / 162.0
    small = np.array(pil.resize((int(round(162 * r)), int(round(120 * r))), Image.Resampling.LANCZOS))
    with torch.no_grad():
        y = O.FORWARDS["johnson"](sd, O.encode(O.to_tensor01(small[None]), "raw_255"))
        o = O.fit_to_content(O.decode(y, "raw_255"), 120, 162)
    ref = O.LabEMA(True, 0.7)(O.to_pil_u8(o.clamp(0, 1))[0])
    got = np.array(Image.open(outp))
    d, within2, dmax = _lsb_report(got, ref)
    assert got.shape == (120, 162, 3) and within2 >= 0.999, (within2, dmax)


@pytest.mark.parametrize("gpus,extra", [(2, []), (3, ["--mask", "MASK", "--smooth_chroma"]),
                                        (2, ["--no-smooth_lightness"]), (2, ["--png_writer", "gpu"])])
def test_multi_gpu_orchestration_gloo_matches_single(tmp_path, monkeypatch, gpus, extra):
    """The --gpus N orchestration (pipeline.py main -> one spawned process per rank, round-robin frames; the LAB
    planes of every frame to rank 0, the ordered EMA there, the smoothed planes back to each frame's owner, which
    merges them, composites the mask, blends and encodes its own frames) with the gloo backend and every rank on
    this box's one GPU: outputs byte-identical to --gpus 1 (frame order and the EMA's sequential state survive the
    sharding), and each rank wrote exactly the frames it stylized."""
    import json
    from neuralstyletransferv1_amd import frames as F
    ck, _ = _ckpt(tmp_path, "johnson", 2)
    frames = synthetic.make_frames(7, 48, 64, seed=90)
    d_in = tmp_path / "in"
    d_in.mkdir()
    for i, f in enumerate(frames):
        Image.fromarray(f).save(d_in / f"frame_{i + 1:04d}.png")
    mask = tmp_path / "mask.png"
    Image.fromarray(((np.indices((48, 64)).sum(0) % 17) * 15).astype(np.uint8)).save(mask)
    extra = [str(mask) if a == "MASK" else a for a in extra]
    outs = {}
    for n in (1, gpus):
        d_out = tmp_path / f"out{n}"
        argv = ["--input_dir", str(d_in), "--output_dir", str(d_out), "--model", ck, "--io_preset", "imagenet_255",
                "--blend", "0.9", "--smooth_alpha", "0.65", "--batch", "2", "--dtype", "bf16",
                "--work_dir", str(tmp_path / f"w{n}")] + extra
        if n > 1:
            wdir = tmp_path / f"written{n}"
            wdir.mkdir()
            monkeypatch.setenv("NST_PIPE_WRITTEN", str(wdir))
            argv += ["--gpus", str(n), "--dist_backend", "gloo", "--dist_timeout", "120"]
        assert P.main(argv) == 0
        outs[n] = [np.array(Image.open(d_out / f"styled_frame_{i + 1:04d}.png")) for i in range(7)]
    for i in range(7):
        assert np.array_equal(outs[1][i], outs[gpus][i]), i
    # each rank encoded exactly its own round-robin shard (groups of `batch` frames per rank)
    groups = F.plan_groups([(48, 64)] * 7, gpus, 2)
    for r in range(gpus):
        got = json.load(open(tmp_path / f"written{gpus}" / f"rank{r}.json"))["written"]
        want = [f"frame_{f + 1:04d}" for g in groups for f in F.shard(g, gpus, r)]
        assert got == want, (r, got, want)


def test_bench_two_ranks_under_torchrun_gloo(tmp_path):
    """The driver's multi-GPU bench command (python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N),
    rehearsed on this one-GPU box: 2 ranks, both on GPU 0 (--device 0), gloo (exchange through host memory), with
    the video pipeline's exchange (--gather: L planes to rank 0, smoothed planes back to the owners).  torchrun is started as a child process (no exec from this process);
    rank 0 prints ONE JSON line with n_gpus 2 and the whole-job frame count.  Scaling itself is not measured here."""
    import json
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "3",
           "--warmup", "1", "--gather", "--dist-backend", "gloo", "--device", "0", "--frame", "960x540",
           "--no-cpu-baseline"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=str(tmp_path),
                       env=dict(os.environ, OMP_NUM_THREADS="4"))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["config"]["dist_backend"] == "gloo"
    assert d["config"]["global_batch"] == 16
    assert d["value"] > 0 and abs(d["value"] - d["config"]["global_batch"] * 3 / (d["ms_per_step"] * 3e-3)) < 1e-3 * d["value"]
    # bench.py's own check of the exchange: the ordered EMA and each owner's final frames equal rank 0's
    # single-rank recomputation (what the driver's N-GPU --gather run reports)
    v = d["gather_verify"]
    assert v["ranks"] == 2 and v["planes_match"] and v["frames_match"], v


def test_bench_gather_self_check_one_rank(tmp_path):
    """bench.py --gather on one rank (no process group): the self-check runs the same exchange schedule (world 1)
    and matches its recomputation."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "2", "--warmup", "1", "--gather",
                        "--frame", "960x540", "--no-cpu-baseline", "--no-fp32", "--no-fp16", "--no-fp16m", "--no-fp32s"],
                       capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    v = d["gather_verify"]
    assert v["ranks"] == 1 and v["planes_match"] and v["frames_match"], v


def test_input_dir_staging_in_memory_jpeg_exif_png(tmp_path):
    """--input_dir staging (pipeline.py:2560-2590) done in memory: a JPEG source is EXIF-uprighted and re-encoded at
    --jpeg_quality before it is stylised, a PNG source is used as its EXIF-upright RGB image.  fp32 CLI without the
    LAB stage vs the oracle on exactly those staged pixels: within +-1 LSB; --keep_staged writes the staged copies
    (decoding them gives the same pixels) and does not change the outputs; a PNG level other than PIL's default
    changes only the file, not the pixels, and so does the fast PNG writer (pngio) against Pillow's."""
    import io
    ck, sd = _ckpt(tmp_path, "johnson", 3)
    frames = synthetic.make_frames(3, 64, 96, seed=77)
    d_in = tmp_path / "in"
    d_in.mkdir()
    staged = []
    for i, f in enumerate(frames):
        im = Image.fromarray(f)
        if i == 1:  # EXIF orientation 6: the reference rotates 270 (upright), so the staged frame is 96 x 64
            exif = Image.Exif()
            exif[0x0112] = 6
            im.save(d_in / f"frame_{i + 1:04d}.jpg", format="JPEG", quality=92, exif=exif)
            up = Image.open(d_in / f"frame_{i + 1:04d}.jpg").convert("RGB").rotate(270, expand=True)
        elif i == 0:
            im.save(d_in / f"frame_{i + 1:04d}.jpg", format="JPEG", quality=92)
            up = Image.open(d_in / f"frame_{i + 1:04d}.jpg").convert("RGB")
        else:
            im.save(d_in / f"frame_{i + 1:04d}.png")
            up = im
        if i < 2:  # the staged JPEG copy at --jpeg_quality 85, decoded
            buf = io.BytesIO()
            up.save(buf, format="JPEG", quality=85)
            buf.seek(0)
            up = Image.open(buf).convert("RGB")
        staged.append(np.array(up))
    outs = {}
    for tag, extra in (("mem", []), ("keep", ["--keep_staged", "--png_compress_level", "1"]),
                       ("pil", ["--png_writer", "pil"]), ("gpu", ["--png_writer", "gpu"])):
        d_out = tmp_path / f"out_{tag}"
        assert P.main(["--input_dir", str(d_in), "--output_dir", str(d_out), "--model", ck, "--io_preset", "imagenet_255",
                       "--pattern", "frame_*", "--no-smooth_lightness", "--batch", "1", "--work_dir",
                       str(tmp_path / f"w_{tag}")] + extra) == 0
        outs[tag] = [np.array(Image.open(d_out / f"styled_frame_{i + 1:04d}.png")) for i in range(3)]
    for i in range(3):
        ref = _oracle_chain([("johnson", sd)], [1.0], [staged[i]], "imagenet_255", smooth=False)[0]
        assert outs["mem"][i].shape == staged[i].shape
        d = np.abs(outs["mem"][i].astype(int) - ref.astype(int))
        print(f"frame {i}: {staged[i].shape}, max |d| {d.max()}")
        assert d.max() <= 1
        assert np.array_equal(outs["mem"][i], outs["keep"][i])
        assert np.array_equal(outs["mem"][i], outs["pil"][i])
        assert np.array_equal(outs["mem"][i], outs["gpu"][i])  # the GPU-built file (csrc/png_enc.hip)
    kept = sorted((tmp_path / "w_keep").rglob("frame_*"))
    assert len(kept) == 3
    for i, p in enumerate(kept):
        assert np.array_equal(np.array(Image.open(p).convert("RGB")), staged[i])


def test_capture_u8_graph_replay_matches_eager():
    """engine.capture_u8 (the bench's HIP-graph step): a replay equals the eager forward bit for bit, and a replay
    after the input buffer is refilled in place stylizes the new frames."""
    from neuralstyletransferv1_amd.engine import capture_u8
    from neuralstyletransferv1_amd.transformer_net import TransformerNet
    net = TransformerNet()
    net.load_state_dict(synthetic.make_state_dict("johnson", 0))
    net = net.cuda().eval()
    net.compute_dtype = "bf16"
    eng = net.engine(torch.device("cuda", 0))
    a = torch.from_numpy(synthetic.make_frames(2, 120, 200, seed=4)).cuda()
    b = torch.from_numpy(synthetic.make_frames(2, 120, 200, seed=5)).cuda()
    frames = a.clone()
    replay, out = capture_u8(eng, frames, "imagenet_255")
    replay()
    torch.cuda.synchronize()
    assert torch.equal(out, eng.stylize_u8(a, "imagenet_255"))
    frames.copy_(b)
    replay()
    torch.cuda.synchronize()
    assert torch.equal(out, eng.stylize_u8(b, "imagenet_255"))
