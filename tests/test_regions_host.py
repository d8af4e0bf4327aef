"""Region-blend compositor, CPU side: the host restatement of region_blend.py's control logic and the
oracle, both pinned against vectors made by the reference module itself (tests/golden/make_golden_regions.py).
"""
import json
import os

import numpy as np
import pytest
import torch

from neuralstyletransferv1_amd import regions as R
from oracle import region_oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")
G = np.load(os.path.join(GOLD, "regions.npz"))
with open(os.path.join(GOLD, "regions.json")) as f:
    META = json.load(f)
H, W = META["H"], META["W"]


def cfg_list(cfgs):
    return [[c.model_indices, c.model_weights, c.scale] for c in cfgs]


def cfgs_from(rows):
    return [R.RegionConfig(list(a), list(b), c) for a, b, c in rows]


@pytest.mark.parametrize("mode", R.MODES)
@pytest.mark.parametrize("count", [4, 5, 7])
def test_hard_masks_bit_exact(mode, count):
    """host draws (random.Random order) + oracle renderer == generate_region_masks(feather=0)"""
    g = R.draw_geometry(H, W, mode, count, 7)
    got = O.masks_from_geometry(g, H, W).numpy().astype(np.uint8)
    assert np.array_equal(got, G[f"masks_{mode}_{count}"])


def test_weighted_voronoi_and_feathers_bit_exact():
    g = R.draw_geometry(H, W, "voronoi", 4, 11, META["region_sizes"])
    assert np.array_equal(O.masks_from_geometry(g, H, W).numpy().astype(np.uint8), G["masks_voronoi_sized"])
    for mode in ("voronoi", "radial", "fractal", "waves"):
        f = O.feather(O.masks_from_geometry(R.draw_geometry(H, W, mode, 4, 3), H, W), 6).numpy()
        assert np.array_equal(f, G[f"fmasks_{mode}"]), mode
    f = O.feather(O.masks_from_geometry(R.draw_geometry(H, W, "grid", 4, 1), H, W), 20).numpy()
    assert np.array_equal(f, G["fmasks_grid_f20"])


def test_assignment_and_configs_match_reference():
    for case in META["assign"]:
        nr, nm, mode, wts, seed, oc = case["args"]
        assert R.assign_models_to_regions(nr, nm, mode, wts, seed, oc) == case["out"], case["args"]
    for case in META["configs"]:
        args = case["args"]
        assert cfg_list(R.parse_region_configs(*args)) == case["out"], args
        assert sorted(R.get_required_scales(*args)) == case["scales"], args


def test_animations_and_specs_match_reference():
    for case in META["blend_anim"]:
        anim = R.parse_blend_animation(case["spec"])
        got = [R.compute_animated_weights([0.5, 0.3, 0.2], f, anim) for f in (0, 1, 17, 45, 89, 200)]
        assert got == case["weights"], case["spec"]
    got = [[a.enabled, a.period, a.waveform, a.phase_offset, a.min_opacity, a.max_opacity]
           for a in R.parse_region_blend_animations("120,sine|60,triangle|static", 5)]
    assert got == META["blend_anim_regions"]
    for case in META["scale_anim"]:
        anim = R.parse_scale_animation(case["spec"])
        assert [R.compute_animated_scale(1.0, f, anim) for f in (0, 5, 15, 31, 59)] == case["scales"], case["spec"]
    for case in META["morph"]:
        m = R.parse_morph_animation(case["spec"])
        assert [m.enabled, m.speed, m.amplitude, m.frequency, m.octaves, m.mode, m.seed] == case["out"], case["spec"]
    got = [R.parse_region_sizes(s, n) for s, n in (("1,1,1,0.2", 4), ("2|1", 5), ("1,2,3,4,5", 3), ("x,1", 2))]
    assert got == META["sizes"]


def test_seed_rules():
    assert R.parse_region_seed(None, True, False) == 42 and R.parse_region_seed(None, False, False) is None
    assert R.parse_region_seed(None, False, True) == 42 and R.parse_region_seed("random", True, False) is None
    assert R.parse_region_seed("fixed", False, False) == 42 and R.parse_region_seed("17", False, False) == 17
    assert R.parse_region_seed("zz", True, False) == 42 and R.parse_region_seed("zz", False, False) is None


def _sources():
    outs = [torch.from_numpy(G["src_outputs"][i]) for i in range(3)]
    orig = torch.from_numpy(G["src_orig_u8"]).permute(2, 0, 1).float().div(255)
    return outs, orig


def test_oracle_composites_bit_exact():
    outs, orig = _sources()
    masks = torch.from_numpy(G["comp_masks"])
    single = [R.RegionConfig([a], [1.0], 1.0) for a in META["comp_assign"]]
    assert np.array_equal(O.composite_adv({1.0: outs}, masks, single, orig, H, W).numpy(), G["comp_out"])
    adv = cfgs_from(META["adv_configs"])
    assert np.array_equal(O.composite_adv({1.0: outs}, masks, adv, orig, H, W).numpy(), G["adv_out"])
    half = [torch.nn.functional.interpolate(o[None], size=(H // 2, W // 2), mode="bilinear",
                                            align_corners=False)[0] for o in outs]
    sc = cfgs_from(META["adv_scaled_configs"])
    assert np.array_equal(O.composite_adv({1.0: outs, 0.5: half}, masks, sc, None, H, W).numpy(), G["adv_scaled_out"])


def test_blend_by_regions_chain_bit_exact():
    """blend_by_regions = draws + masks + feather + assignment + composite (region_blend.py:1690-1787)"""
    outs, orig = _sources()
    for name, mode, count, asg, feather, seed, oc, wts in [
            ("bbr_voronoi", "voronoi", 4, "sequential", 6, 5, 0.0, None),
            ("bbr_diag_orig", "diagonal", 6, "random", 4, 2, 0.4, None),
            ("bbr_weighted", "waves", 5, "weighted", 5, 12, 0.0, [0.2, 0.5, 0.3])]:
        masks = O.feather(O.masks_from_geometry(R.draw_geometry(H, W, mode, count, seed), H, W), feather)
        asn = R.assign_models_to_regions(count, 3, asg, wts, seed, oc)
        cf = [R.RegionConfig([a], [1.0], 1.0) for a in asn]
        got = O.composite_adv({1.0: outs}, masks, cf, orig if oc > 0 else None, H, W).numpy()
        assert np.array_equal(got, G[name]), name
    masks = O.feather(O.masks_from_geometry(R.draw_geometry(H, W, "radial", 4, 6), H, W), 5)
    cf = R.parse_region_configs(4, 3, "random", "A+C|B|O|C:0.9+A:0.1", None, 6, 0.0)
    assert np.array_equal(O.composite_adv({1.0: outs}, masks, cf, orig, H, W).numpy(), G["bbra_spec"])


@pytest.mark.parametrize("case", [0, 1, 2])
def test_crops_plan_and_composite_bit_exact(case):
    outs, orig = _sources()
    c = META["crops"][case]
    masks = O.feather(O.masks_from_geometry(R.draw_geometry(H, W, c["mode"], c["count"], c["seed"]), H, W),
                      c["feather"])
    assert np.array_equal(masks.numpy(), G[f"crops_{case}_masks"])
    cf = R.parse_region_configs(masks.shape[0], 3, "sequential", "A|B+C|C" if case == 0 else None, None, c["seed"], 0.0)
    assert cfg_list(cf) == c["configs"]
    boxes = [O.bbox(masks[k]) for k in range(masks.shape[0])]
    assert [list(b) for b in boxes] == c["bbox"]
    padded = [(max(0, x1 - c["pad"]), max(0, y1 - c["pad"]), min(W, x2 + c["pad"]), min(H, y2 + c["pad"]))
              for x1, y1, x2, y2 in boxes]
    assert [list(b) for b in padded] == c["padded"]
    styled = {}
    for k, ((x1, y1, x2, y2), cfg) in enumerate(zip(padded, cf)):
        for mi in cfg.model_indices:
            if mi >= 0:
                styled.setdefault(mi, {})[k] = outs[mi][:, y1:y2, x1:x2].clone() * 0.9
    anims = R.parse_region_blend_animations("30,triangle", len(cf))
    wts = [R.compute_animated_weights(cfg.model_weights, 7, anims[k]) for k, cfg in enumerate(cf)]
    got = O.composite_crops(styled, padded, cf, masks, orig if c["with_orig"] else None, H, W, wts)
    assert np.array_equal(got.numpy(), G[f"crops_{case}_out"])


def test_feather_taps_match_oracle_kernel():
    for f in (1, 5, 20, 64):
        taps = R.feather_taps(f)
        sigma = f / 3.0
        ks = max(3, int(6 * sigma + 1) | 1)
        assert len(taps) == ks and abs(float(taps.sum()) - 1.0) < 1e-5
    assert R.feather_taps(0) is None


def test_rotation_restatement_properties():
    """cv2 is absent: the warp restatement is parity unpinned; check what holds regardless -- angle 0 is the
    identity, 360 degrees returns the masks, and the rotated set is a partition of unity."""
    masks = O.feather(O.masks_from_geometry(R.draw_geometry(H, W, "voronoi", 4, 3), H, W), 4)
    assert O.rotate(masks, 0) is masks
    r = O.rotate(masks, 30.0)
    s = r.sum(0)
    assert torch.allclose(s, torch.ones_like(s), atol=1e-5)
    back = O.rotate(masks, 360.0)
    assert (back - masks / masks.sum(0).clamp(min=1e-6)).abs().max() < 1e-5


def test_morph_noise_fields_bit_exact():
    fx, fy = O.flow_field(H, W, 3.0, 42, 3 * 1.0 * 0.02)
    assert np.array_equal(np.stack([fx, fy]).astype(np.float32), G["flow_blob"])
    fx, fy = O.flow_field(H, W, 6.0, 142, 5 * 1.5 * 0.02)
    assert np.array_equal(np.stack([fx, fy]).astype(np.float32), G["flow_tentacle_base"])


def test_morph_offsets_follow_numpy_draw_order():
    m = R.MorphAnimation(enabled=True, seed=42)
    off = R.morph_offsets(m, 2)
    rng = np.random.default_rng(142 + 1000)
    assert off[1, 1, 0, 0] == rng.random() * 1000 and off[1, 1, 0, 1] == rng.random() * 1000
    assert off[1, 1, 1, 0] == rng.random() * 1000


def test_morph_restatement_partition_of_unity():
    masks = O.feather(O.masks_from_geometry(R.draw_geometry(H, W, "voronoi", 4, 3), H, W), 4)
    for mode in ("blob", "tentacle", "wave", "pulse"):
        r = O.morph(masks, mode, 1.0, 0.15, 3.0, 42, 5)
        assert torch.allclose(r.sum(0), torch.ones(H, W), atol=1e-5), mode
