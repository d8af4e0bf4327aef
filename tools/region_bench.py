"""Region-blend compositor timing on synthetic 1080p frames, one MI355X.

Two workloads, batch 8 of HBM-resident 1920x1080 uint8 frames, Johnson models in bf16:
  standard  --region_mode voronoi, 4 models, 6 regions, feather 20, original chance 0.25
            (pipeline.py:1720-1839): 4 full-frame forwards + one batched region composite
  optimize  --region_optimize, voronoi, 4 regions, 2 models, padding 64, blend spec "A|B|A+B|O"
            (pipeline.py:1120-1407): per-region crop forwards + the crops composite
Prints one JSON line: ms per step and frames/s of each, the composite kernels' time measured with HIP
events on the stream they run on, and the full-frame composite's input-size rate: all of its inputs
(4 raw f32 sources x 12 B + 6 masks x 4 B + 3 B original + 3 B out = 78 B per pixel) over its time.  The
kernel skips the sources of regions whose mask is 0 at a pixel (exact), so it reads less than that: the
rate is an effective figure, not HBM traffic.
"""
import json
import os
import sys
import time
from types import SimpleNamespace

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neuralstyletransferv1_amd import regions as R, synthetic  # noqa: E402
from neuralstyletransferv1_amd.transformer_net import TransformerNet  # noqa: E402

N, H, W = 8, 1080, 1920
STEPS = int(os.environ.get("REGION_STEPS", "10"))
dev = torch.device("cuda", 0)


def timed(fn, steps):
    for _ in range(2):
        fn()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) / steps * 1e3


def event_ms(fn, steps):
    st = torch.cuda.current_stream(dev)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    a.record(st)
    for _ in range(steps):
        fn()
    b.record(st)
    torch.cuda.synchronize(dev)
    return a.elapsed_time(b) / steps


def args_ns(**kw):
    base = dict(region_mode="voronoi", region_optimize=False, region_count=None, region_sizes=None, region_seed="7",
                region_feather=20, region_assignment="random", region_original=0.0, region_rotate=0.0,
                region_blend_spec=None, region_scales=None, region_padding=64, blend_animate=None,
                blend_animate_regions=None, scale_animate=None, scale_animate_regions=None, region_morph=None,
                blend_models_weights=None)
    base.update(kw)
    return SimpleNamespace(**base)


def main():
    models = []
    for s in range(4):
        net = TransformerNet()
        net.load_state_dict(synthetic.make_state_dict("johnson", seed=s))
        net = net.to(dev).eval()
        net.compute_dtype = "bf16"
        models.append(net)
    frames = torch.from_numpy(synthetic.make_frames(N, H, W, seed=78)).to(dev)
    out = {"workload": "region blend, 1920x1080 batch 8, Johnson bf16", "frames_per_step": N}
    fids = list(range(1, N + 1))

    # ---- standard path ----
    rc = R.RegionCompositor(args_ns(region_count=6, region_original=0.25), dev)
    raws = {}

    def forwards():
        raws["r"] = [R.Source(R.forward_raw(m, frames, "imagenet_255"), "imagenet_255") for m in models]

    def std_step():
        forwards()
        return rc.standard(raws["r"], frames, fids, 4, (H, W))

    out["standard_ms"] = timed(std_step, STEPS)
    out["standard_frames_per_s"] = N * 1e3 / out["standard_ms"]
    forwards()
    comp_ms = event_ms(lambda: rc.standard(raws["r"], frames, fids, 4, (H, W)), STEPS)
    out["standard_composite_ms"] = comp_ms
    out["standard_forwards_ms"] = timed(forwards, STEPS)
    bytes_px = 4 * 12 + 6 * 4 + 3 + 3
    out["composite_all_inputs_gbs"] = N * H * W * bytes_px / (comp_ms * 1e-3) / 1e9
    masks_ms = event_ms(lambda: R.render_masks(R.draw_geometry(H, W, "voronoi", 6, 7), H, W, 20, dev), 5)
    out["masks_ms_voronoi6_feather20"] = masks_ms

    # ---- --region_optimize ----
    ro = R.RegionCompositor(args_ns(region_optimize=True, region_count=4, region_blend_spec="A|B|A+B|O"), dev)
    slots = {0: (models[0], "imagenet_255"), 1: (models[1], "imagenet_255")}
    out["optimize_ms"] = timed(lambda: ro.optimized_frames(slots, frames, fids), STEPS)
    out["optimize_frames_per_s"] = N * 1e3 / out["optimize_ms"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
