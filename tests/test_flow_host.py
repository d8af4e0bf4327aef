"""Temporal stage, CPU side: Pillow's luma formula the GPU kernel uses, and properties of the Farneback
restatement (cv2 is absent: parity unpinned)."""
import numpy as np

from oracle import flow_oracle as FO


def test_luma_formula_matches_pillow():
    rng = np.random.default_rng(1)
    rgb = rng.integers(0, 256, (64, 1024, 3), dtype=np.uint8)
    r, g, b = (rgb[..., i].astype(np.uint32) for i in range(3))
    ours = ((r * 19595 + g * 38470 + b * 7471 + 0x8000) >> 16).astype(np.uint8)
    assert np.array_equal(ours, FO.gray(rgb))


def _texture(h, w, seed=0):
    rng = np.random.default_rng(seed)
    base = FO.gauss_blur(rng.random((h + 40, w + 40)).astype(np.float32), 9, 2.0)
    return ((base - base.min()) / (base.max() - base.min()) * 255).astype(np.float32)


def test_farneback_recovers_translation():
    h, w = 96, 128
    base = _texture(h, w)
    prev = np.clip(base[20:20 + h, 20:20 + w], 0, 255).astype(np.uint8)
    for dx, dy in ((3, 2), (-2, 1), (0, -4)):
        nxt = np.clip(base[20 - dy:20 - dy + h, 20 - dx:20 - dx + w], 0, 255).astype(np.uint8)
        fl = FO.farneback(prev, nxt)[20:-20, 20:-20]
        assert abs(float(np.median(fl[..., 0])) - dx) < 0.05 and abs(float(np.median(fl[..., 1])) - dy) < 0.05


def test_fuse_and_motion_alpha_properties():
    rng = np.random.default_rng(2)
    cur = rng.random((3, 20, 30)).astype(np.float32)
    prev = rng.random((3, 20, 30)).astype(np.float32)
    zero = np.zeros((20, 30, 2), np.float32)
    out = FO.fuse(cur, prev, zero, 0.85)  # zero flow: a plain EMA
    assert np.allclose(out, np.clip(np.float32(0.85) * cur + np.float32(0.15) * prev, 0, 1), atol=1e-6)
    a = FO.motion_alpha(zero, 0.9)
    assert np.allclose(a, 0.9, atol=1e-6)
    big = np.full((20, 30, 2), 50.0, np.float32)
    assert np.allclose(FO.motion_alpha(big, 0.9), 0.4, atol=1e-5)


def test_area_resize_properties():
    """cv2.resize INTER_AREA restated: same size is the identity, 2x2 rounds halves up, fractional cells keep the mean."""
    rng = np.random.default_rng(3)
    g = rng.integers(0, 256, (60, 84), dtype=np.uint8)
    assert np.array_equal(FO.area_resize(g, 60, 84), g)
    s = g.reshape(30, 2, 42, 2).astype(int).sum(axis=(1, 3))
    assert np.array_equal(FO.area_resize(g, 30, 42), ((s + 2) >> 2).astype(np.uint8))
    const = np.full((61, 89), 77, np.uint8)
    assert np.array_equal(FO.area_resize(const, 20, 29), np.full((20, 29), 77, np.uint8))
    small = FO.area_resize(g, 60 // 7, 84 // 5)
    assert abs(float(small.mean()) - float(g.mean())) < 2.0


def test_dis_restatement_recovers_translation():
    from oracle import dis_oracle as DO
    h, w = 128, 160
    base = _texture(h, w, seed=4)
    prev = np.clip(base[20:20 + h, 20:20 + w], 0, 255).astype(np.uint8)
    for dx, dy in ((3, -2), (-4, 1)):
        nxt = np.clip(base[20 - dy:20 - dy + h, 20 - dx:20 - dx + w], 0, 255).astype(np.uint8)
        fl = DO.dis_flow(prev, nxt)[16:-16, 16:-16]
        assert abs(float(np.median(fl[..., 0])) - dx) < 0.2 and abs(float(np.median(fl[..., 1])) - dy) < 0.2
    assert DO.coarsest_scale(1080, 1920) == 6 and DO.coarsest_scale(96, 128) == 2


def test_dis_supported_frame_limits():
    """The host-side size check the flow EMA consults before DIS (temporal.dis_supported; no GPU work): frames
    whose coarsest pyramid level would lie below the finest scale are skipped like the reference's dis.calc
    failures (pipeline.py:1903-1917); 1080p and the usual downscaled sizes run."""
    from neuralstyletransferv1_amd import temporal as T
    assert not T.dis_supported(30, 40)
    assert not T.dis_supported(0, 64)
    for h, w in ((1080, 1920), (540, 960), (270, 480), (96, 128)):
        assert T.dis_supported(h, w), (h, w)
