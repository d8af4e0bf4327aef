"""Temporal stage on the GPU (flow_ops.hip, dis_ops.hip) vs the CPU restatements (oracle/flow_oracle.py,
oracle/dis_oracle.py; cv2 absent: parity unpinned except the luma, which is Pillow's) and end to end through the CLI.

DIS (the reference's default --flow_method): the GPU runs the restatement's fp32 operations in the same order
(its 64-pixel patch sums as the same halving tree); measured, about half of the flow values are identical and the
rest differ by fp32 rounding between the device and numpy in the variational refinement, which the 5 SOR sweeps and
the level-to-level upsampling carry along: max 3.2e-6 px at 96x128, 2.5e-4 px at 270x480 (one pyramid level more).
Bars: 1e-3 px at the 99.9th percentile and 0.05 px at most (room for a search branch that sits on a rounding tie);
translation recovered within 0.15 px (the restatement's own accuracy at finest scale 2 on these textures).

Bars: luma bit-exact vs Pillow; Farneback flow within 2e-3 px of the restatement on >= 99.9 % of pixels (the
same fp32/fp64 operation order; the host exp() of the taps and libm differences can move a fraction of an ulp
through 4 pyramid levels x 3 iterations), translation recovered within 0.05 px; fuse / motion alpha 2e-6."""
import numpy as np
import pytest
import torch
from PIL import Image

from neuralstyletransferv1_amd import pipeline as P
from neuralstyletransferv1_amd import synthetic, temporal as T
from oracle import flow_oracle as FO
from oracle import nst_oracle as NO

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _pair(h, w, dx, dy, seed=0):
    rng = np.random.default_rng(seed)
    base = FO.gauss_blur(rng.random((h + 40, w + 40)).astype(np.float32), 9, 2.0)
    base = (base - base.min()) / (base.max() - base.min()) * 255
    prev = np.clip(base[20:20 + h, 20:20 + w], 0, 255).astype(np.uint8)
    nxt = np.clip(base[20 - dy:20 - dy + h, 20 - dx:20 - dx + w], 0, 255).astype(np.uint8)
    return prev, nxt


def test_gray_bit_exact_vs_pillow():
    fr = synthetic.make_frames(2, 67, 131, seed=4)
    got = T.gray_u8(torch.from_numpy(fr).to(DEV)).cpu().numpy()
    for i in range(2):
        assert np.array_equal(got[i], FO.gray(fr[i]))


@pytest.mark.parametrize("hw", [(72, 96), (135, 240), (270, 480)])
def test_farneback_vs_restatement(hw):
    h, w = hw
    prev, nxt = _pair(h, w, 3, -2)
    got = T.farneback(torch.from_numpy(prev).to(DEV), torch.from_numpy(nxt).to(DEV)).cpu().numpy()
    ref = FO.farneback(prev, nxt)
    d = np.abs(got - ref)
    assert (d > 2e-3).mean() <= 1e-3, float(d.max())
    c = got[20:-20, 20:-20]
    assert abs(float(np.median(c[..., 0])) - 3) < 0.05 and abs(float(np.median(c[..., 1])) + 2) < 0.05


def test_farneback_1080p_translation():
    prev, nxt = _pair(1080, 1920, -5, 4, seed=3)
    fl = T.farneback(torch.from_numpy(prev).to(DEV), torch.from_numpy(nxt).to(DEV)).cpu().numpy()[40:-40, 40:-40]
    assert abs(float(np.median(fl[..., 0])) + 5) < 0.05 and abs(float(np.median(fl[..., 1])) - 4) < 0.05


def test_fuse_and_motion_alpha_vs_restatement():
    rng = np.random.default_rng(5)
    h, w = 64, 80
    cur = rng.random((3, h, w)).astype(np.float32)
    prev = rng.random((3, h, w)).astype(np.float32)
    flow = (rng.random((h, w, 2)).astype(np.float32) - 0.5) * 12
    got = T.fuse(torch.from_numpy(cur).to(DEV), torch.from_numpy(prev).to(DEV), torch.from_numpy(flow).to(DEV), 0.85)
    assert np.abs(got.cpu().numpy() - FO.fuse(cur, prev, flow, 0.85)).max() <= 2e-6
    a = T.motion_alpha(torch.from_numpy(flow).to(DEV), 0.9).cpu().numpy()
    assert np.abs(a - FO.motion_alpha(flow, 0.9)).max() <= 2e-6


def test_fuse_non_finite_and_huge_flow():
    """A degenerate flow (NaN, +-inf, 1e30) must not index outside the previous frame: the remap coordinates
    are clamped to [-2w, 3w] x [-2h, 3h] before the 1/32-pixel fixed point (cv2's saturate_cast), NaN taken
    to the low end; the output stays finite and equals the restatement."""
    rng = np.random.default_rng(6)
    h, w = 40, 56
    cur = rng.random((3, h, w)).astype(np.float32)
    prev = rng.random((3, h, w)).astype(np.float32)
    flow = (rng.random((h, w, 2)).astype(np.float32) - 0.5) * 6
    flow[3, 5] = np.nan
    flow[7, 9, 0] = np.inf
    flow[8, 10, 1] = -np.inf
    flow[11, 12] = 1e30
    flow[13, 14] = -1e30
    got = T.fuse(torch.from_numpy(cur).to(DEV), torch.from_numpy(prev).to(DEV), torch.from_numpy(flow).to(DEV), 0.7)
    got = got.cpu().numpy()
    assert np.isfinite(got).all()
    assert np.abs(got - FO.fuse(cur, prev, flow, 0.7)).max() <= 2e-6


def test_cli_flow_ema_motion_blend_vs_oracle(tmp_path):
    """pipeline.py:1884-2094 per frame: model -> out01 -> flow EMA (Farneback on Pillow luma) -> ToPILImage ->
    LAB EMA -> motion-adaptive blend with the original (--blend 0.9), fp32."""
    sd = synthetic.make_state_dict("johnson", 3)
    ck = tmp_path / "m.pth"
    torch.save(sd, ck)
    h, w = 64, 96
    frames = []
    base = synthetic.make_frames(1, h + 16, w + 16, seed=50)[0]
    for i in range(3):  # a pan: the content moves 2 px right, 1 px down per frame
        frames.append(np.ascontiguousarray(base[8 - i:8 - i + h, 8 - 2 * i:8 - 2 * i + w]))
    d_in, d_out = tmp_path / "in", tmp_path / "out"
    d_in.mkdir()
    for i, f in enumerate(frames):
        Image.fromarray(f).save(d_in / f"frame_{i + 1:04d}.png")
    assert P.main(["--input_dir", str(d_in), "--output_dir", str(d_out), "--work_dir", str(tmp_path / "w"), "--model",
                   str(ck), "--io_preset", "imagenet_255", "--flow_ema", "--flow_method", "farneback", "--flow_alpha",
                   "0.8", "--motion_blend", "--blend", "0.9", "--batch", "2"]) == 0
    ema = NO.LabEMA(True, 0.7)
    prev_gray = prev01 = None
    for i, fr in enumerate(frames):
        x01 = NO.to_tensor01(fr[None])
        with torch.no_grad():
            out01 = NO.decode(NO.FORWARDS["johnson"](sd, NO.encode(x01, "imagenet_255")), "imagenet_255")[0].numpy()
        g = FO.gray(fr)
        flow = None
        if prev_gray is not None:
            flow = FO.farneback(prev_gray, g)
            out01 = FO.fuse(out01, prev01, flow, 0.8)
        prev_gray, prev01 = g, out01
        u8 = ema((torch.from_numpy(out01)[None].mul(255).byte().permute(0, 2, 3, 1).numpy())[0])
        o01 = fr.astype(np.float32) / 255
        s01 = u8.astype(np.float32) / 255
        if flow is not None:
            a = FO.motion_alpha(flow, 0.9)[..., None]
            ref = np.clip(a * s01 + (1 - a) * o01, 0, 1)
        else:
            ref = np.clip(np.float32(0.9) * s01 + np.float32(0.1) * o01, 0, 1)
        ref = (ref * 255).astype(np.uint8)
        got = np.array(Image.open(d_out / f"styled_frame_{i + 1:04d}.png"))
        dd = np.abs(got.astype(int) - ref.astype(int))
        assert (dd > 1).mean() <= 0.005, f"frame {i}: {(dd > 1).mean():.4%} > 1 LSB (max {dd.max()})"


def test_flow_downscale_vs_restatement():
    prev, nxt = _pair(144, 256, 4, 2, seed=7)
    for ds in (2, 4):
        g = T.downscale_gray(torch.from_numpy(prev).to(DEV), ds).cpu().numpy()
        assert np.array_equal(g, FO.area_down(prev, ds))
    fs = T.FlowSmoother(True, 0.8, 2, "farneback")
    a = torch.rand(3, 144, 256, device=DEV)
    fr0 = np.repeat(prev[..., None], 3, axis=2)
    fr1 = np.repeat(nxt[..., None], 3, axis=2)
    fs(a, torch.from_numpy(fr0).to(DEV))
    fs(a, torch.from_numpy(fr1).to(DEV))
    got = fs.last_flow.cpu().numpy()
    ref = FO.farneback_downscaled(FO.gray(fr0), FO.gray(fr1), 2)
    d = np.abs(got - ref)
    assert (d > 4e-3).mean() <= 1e-3, float(d.max())
    c = got[24:-24, 24:-24]
    assert abs(float(np.median(c[..., 0])) - 4) < 0.1 and abs(float(np.median(c[..., 1])) - 2) < 0.1


def _dis_pairs(n, h, w, seed=0):
    moves = [(3, -2), (-5, 4), (2, 3), (-1, -6)]
    ps, ns = [], []
    for k in range(n):
        p, q = _pair(h, w, *moves[k % 4], seed=seed + k)
        ps.append(p)
        ns.append(q)
    return np.stack(ps), np.stack(ns), [moves[k % 4] for k in range(n)]


@pytest.mark.parametrize("hw", [(96, 128), (256, 320), (270, 480)])
def test_dis_vs_restatement(hw):
    from oracle import dis_oracle as DO
    h, w = hw
    prev, nxt, moves = _dis_pairs(2, h, w)
    got = T.dis(torch.from_numpy(prev).to(DEV), torch.from_numpy(nxt).to(DEV)).cpu().numpy()
    for k in range(2):
        ref = DO.dis_flow(prev[k], nxt[k])
        d = np.abs(got[k] - ref)
        same = float((d == 0).mean())
        print(hw, k, f"identical {same:.5f}, max |d| {d.max():.3e}, p99.9 {np.quantile(d, 0.999):.3e}")
        assert np.quantile(d, 0.999) <= 1e-3 and d.max() <= 0.05, (same, float(d.max()))
        c = got[k][16:-16, 16:-16]
        dx, dy = moves[k]
        assert abs(float(np.median(c[..., 0])) - dx) < 0.15 and abs(float(np.median(c[..., 1])) - dy) < 0.15


def test_dis_batch_equals_single_and_1080p_translation():
    prev, nxt, moves = _dis_pairs(3, 1080, 1920, seed=11)
    pd, nd = torch.from_numpy(prev).to(DEV), torch.from_numpy(nxt).to(DEV)
    batch = T.dis(pd, nd).cpu().numpy()
    for k in range(3):
        one = T.dis(pd[k], nd[k]).cpu().numpy()
        assert np.array_equal(one, batch[k]), k
        c = one[64:-64, 64:-64]
        dx, dy = moves[k]
        print("1080p", k, np.median(c[..., 0]), np.median(c[..., 1]))
        assert abs(float(np.median(c[..., 0])) - dx) < 0.15 and abs(float(np.median(c[..., 1])) - dy) < 0.15


def test_dis_rejects_tiny_frames():
    from neuralstyletransferv1_amd._lib import NstError
    g = torch.zeros((40, 60), dtype=torch.uint8, device=DEV)
    with pytest.raises(NstError, match="too small"):
        T.dis(g, g)


@pytest.mark.parametrize("geom", [((144, 256), (48, 85)), ((720, 1280), (240, 426)), ((97, 131), (97 // 2, 131 // 2)),
                                  ((270, 480), (135, 240)), ((135, 240), (67, 120)), ((50, 70), (50, 70))])
def test_area_resize_vs_restatement(geom):
    """cv2.resize INTER_AREA (the DIS pyramid, --flow_downscale's floored sizes): integer and fractional cells."""
    (h, w), (oh, ow) = geom
    rng = np.random.default_rng(h + w)
    img = rng.integers(0, 256, (2, h, w), dtype=np.uint8)
    out = torch.empty((2, oh, ow), dtype=torch.uint8, device=DEV)
    from neuralstyletransferv1_amd._lib import check, lib, stream_ptr
    src = torch.from_numpy(img).to(DEV)
    check(lib().nst_resize_area_u8(src.data_ptr(), 2, h, w, 1, out.data_ptr(), oh, ow, stream_ptr(DEV)), "area")
    got = out.cpu().numpy()
    for k in range(2):
        assert np.array_equal(got[k], FO.area_resize(img[k], oh, ow)), (geom, k)


def test_cli_flow_ema_default_dis_vs_oracle(tmp_path):
    """--flow_ema with the reference's default --flow_method (dis) through the CLI, fp32, against the oracle chain
    with the DIS restatement (and the 2nd/3rd frames' flows equal to the restatement's)."""
    from oracle import dis_oracle as DO
    sd = synthetic.make_state_dict("johnson", 4)
    ck = tmp_path / "m.pth"
    torch.save(sd, ck)
    h, w = 96, 128
    base = synthetic.make_frames(1, h + 16, w + 16, seed=51)[0]
    frames = [np.ascontiguousarray(base[8 - i:8 - i + h, 8 - 2 * i:8 - 2 * i + w]) for i in range(3)]
    d_in, d_out = tmp_path / "in", tmp_path / "out"
    d_in.mkdir()
    for i, f in enumerate(frames):
        Image.fromarray(f).save(d_in / f"frame_{i + 1:04d}.png")
    assert P.main(["--input_dir", str(d_in), "--output_dir", str(d_out), "--work_dir", str(tmp_path / "w"), "--model",
                   str(ck), "--io_preset", "imagenet_255", "--flow_ema", "--flow_alpha", "0.8", "--batch", "3"]) == 0
    ema = NO.LabEMA(True, 0.7)
    prev_gray = prev01 = None
    for i, fr in enumerate(frames):
        x01 = NO.to_tensor01(fr[None])
        with torch.no_grad():
            out01 = NO.decode(NO.FORWARDS["johnson"](sd, NO.encode(x01, "imagenet_255")), "imagenet_255")[0].numpy()
        g = FO.gray(fr)
        if prev_gray is not None:
            out01 = FO.fuse(out01, prev01, DO.dis_flow(prev_gray, g), 0.8)
        prev_gray, prev01 = g, out01
        ref = ema((torch.from_numpy(out01)[None].mul(255).byte().permute(0, 2, 3, 1).numpy())[0])
        got = np.array(Image.open(d_out / f"styled_frame_{i + 1:04d}.png"))
        dd = np.abs(got.astype(int) - ref.astype(int))
        print(i, "max", dd.max(), "> 1 LSB", (dd > 1).mean())
        assert (dd > 1).mean() <= 0.005, f"frame {i}: {(dd > 1).mean():.4%} > 1 LSB (max {dd.max()})"


def test_cli_flow_downscale_non_divisor(tmp_path):
    """--flow_downscale 3 on frames it does not divide (pipeline.py:1886-1889 floors W0 // 3, H0 // 3): runs and
    matches the restatement chain's flow."""
    from oracle import dis_oracle as DO
    h, w = 280, 383
    prev, nxt = _pair(h, w, 6, -3, seed=9)
    fs = T.FlowSmoother(True, 0.8, 3, "dis")
    a = torch.rand(3, h, w, device=DEV)
    fr0 = np.repeat(prev[..., None], 3, axis=2)
    fr1 = np.repeat(nxt[..., None], 3, axis=2)
    fs(a, torch.from_numpy(fr0).to(DEV))
    fs(a, torch.from_numpy(fr1).to(DEV))
    got = fs.last_flow.cpu().numpy()
    g0, g1 = FO.gray(fr0), FO.gray(fr1)
    small = DO.dis_flow(FO.area_down(g0, 3), FO.area_down(g1, 3))
    ref = FO.resize_lin(small, h, w, 3.0)
    d = np.abs(got - ref)
    print("ds3", (d == 0).mean(), d.max())
    assert np.quantile(d, 0.999) <= 1e-3 and d.max() <= 0.05
    # no translation check here: DIS PRESET_FAST on the 93 x 127 reduced gray does not recover the 2 x -1 px
    # shift (its finest scale is 2, so 4-px patches on a ~46 x 63 grid); the restatement's field is the same


def test_cli_flow_ema_dis_small_frames_pass_through(tmp_path):
    """--flow_ema (DIS) on frames too small for DIS PRESET_FAST (80 x 60 with --flow_downscale 2 -> 40 x 30 grays):
    the reference's dis.calc try/except skips the flow for the frame (pipeline.py:1903-1917), so every frame is
    written unfused, equal to the same run without --flow_ema."""
    sd = synthetic.make_state_dict("johnson", 5)
    ck = tmp_path / "m.pth"
    torch.save(sd, ck)
    d_in = tmp_path / "in"
    d_in.mkdir()
    for i, f in enumerate(synthetic.make_frames(3, 60, 80, seed=52)):
        Image.fromarray(f).save(d_in / f"frame_{i + 1:04d}.png")
    assert not T.dis_supported(30, 40)
    outs = {}
    for tag, extra in (("flow", ["--flow_ema", "--flow_downscale", "2"]), ("plain", [])):
        d_out = tmp_path / f"out_{tag}"
        assert P.main(["--input_dir", str(d_in), "--output_dir", str(d_out), "--work_dir", str(tmp_path / f"w_{tag}"),
                       "--model", str(ck), "--io_preset", "imagenet_255", "--batch", "2"] + extra) == 0
        outs[tag] = [np.array(Image.open(d_out / f"styled_frame_{i + 1:04d}.png")) for i in range(3)]
    for a, b in zip(outs["flow"], outs["plain"]):
        d = np.abs(a.astype(int) - b.astype(int))
        print("differing values", int((d > 0).sum()), "max", int(d.max()))
        assert d.max() <= 1  # the --flow_ema path truncates the fp32 out01 on its own kernel (same arithmetic)
