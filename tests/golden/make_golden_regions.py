"""Generate tests/golden/regions.npz + regions.json from the REFERENCE region_blend.py (build container
only; /root/reference does not exist on the GPU box and nothing at test time reads it).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_regions.py

region_blend.py imports cv2 at module level (region_blend.py:14) but cv2 is not installed here.  Only
the functions that never touch cv2 are called below (mask generators, feather = torch conv2d, model
assignment, config / animation parsing, the composites, crops, the numpy noise fields of the morph
animation), so the module is imported with an EMPTY placeholder module under the name cv2: any call
that did reach cv2 would raise AttributeError instead of producing a vector.  rotate_mask (cv2.warpAffine)
and warp_mask_organic's cv2.remap are therefore NOT pinned here (parity unpinned).

Stored (all seeded; sizes small so the oracle and the GPU tests finish in seconds):
  masks_<mode>_<count>   hard masks (feather 0) of generate_region_masks, uint8 0/1 [K,H,W]
  fmasks_<mode>          feathered masks (feather 6), float32 [K,H,W]
  comp_* / adv_* / bbr_* / crops_*   composite outputs, float32 [3,H,W], with their inputs
  regions.json           assignments, configs, animation weights, bboxes (host-logic vectors)
"""
from __future__ import annotations

import json
import os
import random
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("NST_REFERENCE", "/root/reference")

H, W = 45, 80
MODES = ["grid", "diagonal", "voronoi", "fractal", "radial", "waves", "spiral", "concentric", "random"]


def load_reference():
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))  # placeholder: see the module docstring
    sys.path.insert(0, REF)
    import region_blend as rb  # noqa: E402
    return rb


def main():
    rb = load_reference()
    torch.manual_seed(0)
    arrays, meta = {}, {"H": H, "W": W, "torch": torch.__version__, "numpy": np.__version__}

    # ---- mask generators (region_blend.py:109-516, 925-980) ----
    for mode in MODES:
        for count in (4, 5, 7):
            ms = rb.generate_region_masks(H, W, mode, count, seed=7, feather=0)
            arrays[f"masks_{mode}_{count}"] = torch.cat(ms, 0)[:, 0].numpy().astype(np.uint8)
    sizes = rb.parse_region_sizes("1,1,1,0.2", 4)
    meta["region_sizes"] = sizes
    arrays["masks_voronoi_sized"] = torch.cat(rb.generate_region_masks(H, W, "voronoi", 4, 11, 0, sizes), 0)[:, 0] \
        .numpy().astype(np.uint8)
    for mode in ("voronoi", "radial", "fractal", "waves"):
        ms = rb.generate_region_masks(H, W, mode, 4, seed=3, feather=6)
        arrays[f"fmasks_{mode}"] = torch.cat(ms, 0)[:, 0].numpy().astype(np.float32)
    # a large feather relative to the frame (kernel 41 on a 45-row frame: reflect padding near its limit)
    arrays["fmasks_grid_f20"] = torch.cat(rb.generate_region_masks(H, W, "grid", 4, 1, 20), 0)[:, 0].numpy()

    # ---- host logic: assignment / configs / animations ----
    meta["assign"] = []
    for (nr, nm, mode, wts, seed, oc) in [(6, 3, "sequential", None, 1, 0.0), (6, 3, "sequential", None, 1, 0.3),
                                          (8, 4, "random", None, 5, 0.0), (8, 4, "random", None, 5, 0.4),
                                          (8, 3, "weighted", [0.5, 0.3, 0.2], 9, 0.0),
                                          (8, 3, "weighted", [0.5, 0.3, 0.2], 9, 0.25)]:
        meta["assign"].append({"args": [nr, nm, mode, wts, seed, oc],
                               "out": rb.assign_models_to_regions(nr, nm, mode, wts, seed, oc)})
    meta["configs"] = []
    for (nr, nm, asg, spec, scales, seed, oc) in [(4, 3, "sequential", None, None, 2, 0.0),
                                                  (5, 3, "random", None, "1.0,0.5", 4, 0.3),
                                                  (6, 4, "random", "A+B|C:0.7+D:0.3|O|B", "1.0|0.5|0.25", 8, 0.0),
                                                  (3, 2, "sequential", "a:0.2+b+O", None, 1, 0.0),
                                                  (4, 8, "sequential", "A|H|1+2|ORIGINAL", "0.5", 3, 0.0)]:
        cf = rb.parse_region_configs(nr, nm, asg, spec, scales, seed, oc)
        meta["configs"].append({"args": [nr, nm, asg, spec, scales, seed, oc],
                                "out": [[c.model_indices, c.model_weights, c.scale] for c in cf],
                                "scales": sorted(rb.get_required_scales(nr, nm, asg, spec, scales, seed, oc))})
    meta["blend_anim"] = []
    for spec in ["120", "60,triangle", "90,sine,45", "120,sine,0,0.2,0.8", "40,sawtooth", "40,sawtooth_down",
                 "30,square,90", "static", "0", "7,bogus"]:
        anim = rb.parse_blend_animation(spec)
        ws = [rb.compute_animated_weights([0.5, 0.3, 0.2], f, anim) for f in (0, 1, 17, 45, 89, 200)]
        meta["blend_anim"].append({"spec": spec, "weights": ws})
    meta["blend_anim_regions"] = [[a.enabled, a.period, a.waveform, a.phase_offset, a.min_opacity, a.max_opacity]
                                  for a in rb.parse_region_blend_animations("120,sine|60,triangle|static", 5)]
    meta["scale_anim"] = []
    for spec in ["60", "60,triangle,0,0.3,0.8", "90,sine,45", "static"]:
        anim = rb.parse_scale_animation(spec)
        meta["scale_anim"].append({"spec": spec, "scales": [rb.compute_animated_scale(1.0, f, anim)
                                                            for f in (0, 5, 15, 31, 59)]})
    meta["morph"] = []
    for spec in ["blob", "tentacle", "1.5,0.2,4.0,blob", "2.0,0.1,3.0,tentacle", "2.5,0.3", "1.2", "wavy", "off"]:
        m = rb.parse_morph_animation(spec)
        meta["morph"].append({"spec": spec, "out": [m.enabled, m.speed, m.amplitude, m.frequency, m.octaves,
                                                    m.mode, m.seed]})
    meta["sizes"] = [rb.parse_region_sizes(s, n) for s, n in (("1,1,1,0.2", 4), ("2|1", 5), ("1,2,3,4,5", 3),
                                                               ("x,1", 2))]

    # ---- morph noise fields (numpy only; region_blend.py:604-667) ----
    fx, fy = rb._generate_flow_field(H, W, 3.0, 42, 3 * 1.0 * 0.02)
    arrays["flow_blob"] = np.stack([fx, fy]).astype(np.float32)
    fx, fy = rb._generate_flow_field(H, W, 6.0, 142, 5 * 1.5 * 0.02)
    arrays["flow_tentacle_base"] = np.stack([fx, fy]).astype(np.float32)

    # ---- composites ----
    g = torch.Generator().manual_seed(1)
    outs = [torch.rand(3, H, W, generator=g) for _ in range(3)]
    orig_u8 = (torch.rand(H, W, 3, generator=g) * 255).to(torch.uint8)
    orig = orig_u8.permute(2, 0, 1).float().div(255)
    arrays["src_outputs"] = torch.stack(outs).numpy()
    arrays["src_orig_u8"] = orig_u8.numpy()
    masks = rb.generate_region_masks(H, W, "voronoi", 5, seed=3, feather=6)
    assign = [0, 2, -1, 1, 0]
    arrays["comp_masks"] = torch.cat(masks, 0)[:, 0].numpy()
    arrays["comp_out"] = rb.composite_regions(outs, masks, assign, orig).numpy()
    meta["comp_assign"] = assign
    cfgs = rb.parse_region_configs(5, 3, "random", "A:0.6+B|C|O+A|B", None, 4, 0.0)
    arrays["adv_out"] = rb.composite_regions_advanced({1.0: outs}, masks, cfgs, orig, H, W).numpy()
    meta["adv_configs"] = [[c.model_indices, c.model_weights, c.scale] for c in cfgs]
    # scales: the pipeline's simulated low-res outputs (pipeline.py:1786-1796) then the composite's upsample
    half = [torch.nn.functional.interpolate(o[None], size=(int(H * 0.5), int(W * 0.5)), mode="bilinear",
                                            align_corners=False)[0] for o in outs]
    cfgs_s = rb.parse_region_configs(5, 3, "sequential", None, "1.0,0.5", 4, 0.0)
    arrays["adv_scaled_out"] = rb.composite_regions_advanced({1.0: outs, 0.5: half}, masks, cfgs_s, None, H, W).numpy()
    meta["adv_scaled_configs"] = [[c.model_indices, c.model_weights, c.scale] for c in cfgs_s]
    for name, kw in [("bbr_voronoi", dict(mode="voronoi", region_count=4, assignment="sequential", feather=6, seed=5)),
                     ("bbr_diag_orig", dict(mode="diagonal", region_count=6, assignment="random", feather=4, seed=2,
                                            original=orig, original_chance=0.4)),
                     ("bbr_weighted", dict(mode="waves", region_count=5, assignment="weighted",
                                           weights=[0.2, 0.5, 0.3], feather=5, seed=12))]:
        arrays[name] = rb.blend_by_regions(outs, H, W, **kw).numpy()
    arrays["bbra_spec"] = rb.blend_by_regions_advanced({1.0: outs}, H, W, mode="radial", region_count=4,
                                                       assignment="random", blend_spec="A+C|B|O|C:0.9+A:0.1",
                                                       feather=5, seed=6, original=orig).numpy()

    # ---- crops (region_blend.py:1969-2294) ----
    meta["crops"] = []
    for case, (mode, count, seed, feather, pad, with_orig) in enumerate([("voronoi", 4, 3, 6, 8, True),
                                                                        ("grid", 3, 1, 0, 4, False),
                                                                        ("fractal", 5, 9, 3, 6, False)]):
        ms = rb.generate_region_masks(H, W, mode, count, seed, feather)
        cf = rb.parse_region_configs(len(ms), 3, "sequential", "A|B+C|C" if case == 0 else None, None, seed, 0.0)
        crops = rb.prepare_region_crops(ms, cf, H, W, pad)
        styled = {}
        for c in crops:
            x1, y1, x2, y2 = c.padded_bbox
            for mi in c.config.model_indices:
                if mi >= 0:
                    styled.setdefault(mi, {})[c.region_idx] = outs[mi][:, y1:y2, x1:x2].clone() * 0.9
        out = rb.composite_from_crops(styled, crops, orig if with_orig else None, H, W, frame_idx=7,
                                      blend_animations=rb.parse_region_blend_animations("30,triangle", len(crops)))
        arrays[f"crops_{case}_masks"] = torch.cat(ms, 0)[:, 0].numpy()
        arrays[f"crops_{case}_out"] = out.numpy()
        meta["crops"].append({"mode": mode, "count": count, "seed": seed, "feather": feather, "pad": pad,
                              "with_orig": with_orig, "bbox": [list(c.bbox) for c in crops],
                              "padded": [list(c.padded_bbox) for c in crops],
                              "configs": [[c.config.model_indices, c.config.model_weights, c.config.scale]
                                          for c in crops],
                              "needed": rb.get_models_needed_for_regions(crops),
                              "coverage": rb.compute_crop_coverage(crops, H, W)})

    np.savez_compressed(os.path.join(HERE, "regions.npz"), **arrays)
    with open(os.path.join(HERE, "regions.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote", len(arrays), "arrays")


if __name__ == "__main__":
    random.seed(0)
    main()
