"""configs[4] timing: DeepLab v3+ mask + stylization + mask composite on synthetic 1080p frames, one MI355X.

Step = one batch of 8 HBM-resident 1920x1080 uint8 frames through
  MaskEngine (Pillow-exact LANCZOS to the 256-px working size -> DeepLab v3+ ResNet-101 -> argmax ->
  class selection -> close 5x5 -> blur (feather 3) -> INTER_LINEAR back to 1080p)   [sky_swap.py:271-366]
  + Johnson stylization (bf16)                                                        [pipeline.py:1445-1519]
  + mask composite, keep mode (alpha = m / 255)                                        [pipeline.py:1984-2048]
Prints one JSON line: frames/s of the whole step, ms of each stage, and the DeepLab forward's algorithmic
TFLOP/s at the working size and at full 1080p (--resolution 0), which is where conv_gemm is MFMA-bound."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neuralstyletransferv1_amd import deeplab, synthetic  # noqa: E402
from neuralstyletransferv1_amd.postproc import blend_frames  # noqa: E402
from neuralstyletransferv1_amd.transformer_net import TransformerNet  # noqa: E402

N, H, W = 8, 1080, 1920
STEPS = int(os.environ.get("SEG_STEPS", "10"))
dev = torch.device("cuda", 0)


def deeplab_gflop(h, w, nc=19):
    """2 * MACs of every conv of the OS16 ResNet-101 DeepLab v3+ at input h x w."""
    def ext(v, k, s, d, p):
        return (v + 2 * p - d * (k - 1) - 1) // s + 1
    macs = 0
    h2, w2 = ext(h, 7, 2, 1, 3), ext(w, 7, 2, 1, 3)
    macs += h2 * w2 * 64 * 147
    hh, ww = ext(h2, 3, 2, 1, 1), ext(w2, 3, 2, 1, 1)
    h4, w4 = hh, ww
    inpl = 64
    for li, (nb, planes, stride) in enumerate(((3, 64, 1), (4, 128, 2), (23, 256, 2), (3, 512, 1))):
        for i in range(nb):
            s = stride if i == 0 else 1
            d = 1 if li < 3 else 2 * (1, 2, 4)[i]
            ho, wo = ext(hh, 3, s, d, d), ext(ww, 3, s, d, d)
            macs += hh * ww * inpl * planes + ho * wo * planes * planes * 9 + ho * wo * planes * planes * 4
            if i == 0:
                macs += ho * wo * inpl * planes * 4
            inpl = planes * 4
            hh, ww = ho, wo
    macs += hh * ww * 2048 * 256 * (1 + 9 * 3) + 2048 * 256 + hh * ww * 1280 * 256
    macs += h4 * w4 * (256 * 48 + 304 * 256 * 9 + 256 * 256 * 9 + 256 * nc)
    return 2 * macs / 1e9


def timed(fn, steps):
    for _ in range(2):
        fn()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) / steps * 1e3


# the mask program's dtype in the configs[4] step: fp32s, the fastest mode holding the fp32 bars against the reference
# logits (sky_swap.py --dtype fp32s; the CLI's default is exact fp32)
MASK_DT = os.environ.get("SEG_MASK_DT", "fp32s")


def main():
    model = deeplab.DeepLab(num_classes=19)
    model.load_state_dict(deeplab.make_state_dict(19, 0))
    model = model.eval().to(dev)
    net = TransformerNet()
    net.load_state_dict(synthetic.make_state_dict("johnson", seed=0))
    net = net.to(dev).eval()
    net.compute_dtype = "bf16"
    eng = net.engine(dev)
    frames = torch.from_numpy(synthetic.make_frames(N, H, W, seed=77)).to(dev)
    ids = [10]  # Cityscapes "sky" (sky_swap.py:83)
    out = {"workload": "configs[4]: DeepLab v3+ mask (256-px working size) + Johnson stylization + mask composite, "
                       "1920x1080 batch 8, bf16", "frames_per_step": N}
    res = {}
    for dtype in os.environ.get("SEG_DTYPES", "bf16,fp16,fp32,fp32s").split(","):
        me = deeplab.MaskEngine(model, dev, resolution=256, dtype=dtype)
        res[dtype] = timed(lambda: me.masks(frames, ids, feather_px=3), STEPS)
    me = deeplab.MaskEngine(model, dev, resolution=256, dtype=MASK_DT)
    hw = deeplab.working_size(W, H, 256)
    work = me._resampler("lanczos", H, W, hw[1], hw[0])(frames)
    seg = model.engine(dev, MASK_DT)
    fwd_ms = timed(lambda: seg.run(work, logits=False, pred=True), STEPS)
    lanczos_ms = timed(lambda: me._resampler("lanczos", H, W, hw[1], hw[0])(frames), STEPS)
    g_work = deeplab_gflop(hw[1], hw[0]) * N
    out.update({"mask_dtype": MASK_DT, **{f"mask_ms_{d}": round(t, 3) for d, t in res.items()},
                "lanczos_ms": round(lanczos_ms, 3), "deeplab_fwd_ms": round(fwd_ms, 3),
                "deeplab_gflop_per_batch": round(g_work, 2),
                "deeplab_tflops_working_size": round(g_work / fwd_ms, 1)})
    # full-resolution DeepLab (sky_swap --resolution 0): large GEMMs, two frames
    big = frames[:2].contiguous()
    full_ms = timed(lambda: seg.run(big, logits=False, pred=True), max(3, STEPS // 3))
    g_full = deeplab_gflop(H, W) * 2
    out.update({"deeplab_fullres_ms_2frames": round(full_ms, 3), "deeplab_fullres_gflop_2frames": round(g_full, 1),
                "deeplab_fullres_tflops": round(g_full / full_ms, 1)})
    # the whole configs[4] step
    def step():
        m = me.masks(frames, ids, feather_px=3)
        st = eng.stylize_u8(frames, "imagenet_255")
        return blend_frames(st, frames, 1.0, m, "keep")
    ms = timed(step, STEPS)
    styl_ms = timed(lambda: eng.stylize_u8(frames, "imagenet_255"), STEPS)
    out.update({"step_ms": round(ms, 3), "frames_per_s": round(N / ms * 1e3, 1), "stylize_ms": round(styl_ms, 3),
                "mask_share": round(res[MASK_DT] / ms, 3),
                # the step with each mask dtype: its mask time / (that + the rest of the step)
                "mask_share_by_dtype": {d: round(t / (ms - res[MASK_DT] + t), 3) for d, t in res.items()}})
    # the same step with the mask program on a second HIP stream beside the stylization (independent until the
    # composite): DeepLab's small GEMMs leave most CUs idle, and the stylization's kernels fill them
    side = torch.cuda.Stream(dev)

    def step_overlap():
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            m = me.masks(frames, ids, feather_px=3)
        st = eng.stylize_u8(frames, "imagenet_255")
        torch.cuda.current_stream(dev).wait_stream(side)
        m.record_stream(torch.cuda.current_stream(dev))
        return blend_frames(st, frames, 1.0, m, "keep")
    ref_out = step()
    ov_out = step_overlap()
    torch.cuda.synchronize(dev)
    ov_ms = timed(step_overlap, STEPS)
    out.update({"step_ms_overlap": round(ov_ms, 3), "frames_per_s_overlap": round(N / ov_ms * 1e3, 1),
                # the part of the overlapped step the mask adds beyond the stylization alone
                "mask_exposed_share_overlap": round(max(0.0, ov_ms - styl_ms) / ov_ms, 3),
                "overlap_identical": bool(torch.equal(ref_out, ov_out))})
    # a larger mask batch: one DeepLab run per `mb` frames (the masks of mb / 8 stylization steps), which amortises
    # the latency-bound ResNet layer3 GEMMs (1,152 output pixels per 8 frames); the step below runs one mask call
    # and mb / 8 stylize + composite steps, reported per 8 frames
    mbs = [int(v) for v in os.environ.get("SEG_MASK_BATCHES", "32,64,128").split(",") if v]
    for mb in mbs:
        big = torch.cat([frames] * (mb // N)).contiguous()
        mb_ms = timed(lambda: me.masks(big, ids, feather_px=3), max(3, STEPS // 2))
        k = mb // N

        def step_mb():
            m = me.masks(big, ids, feather_px=3)
            outs = []
            for j in range(k):
                st = eng.stylize_u8(frames, "imagenet_255")
                outs.append(blend_frames(st, frames, 1.0, m[j * N:(j + 1) * N], "keep"))
            return outs
        ms_mb = timed(step_mb, max(3, STEPS // 2)) / k
        same = torch.equal(step_mb()[0], ref_out)
        out[f"mask_batch_{mb}"] = {"mask_ms_per_8_frames": round(mb_ms * N / mb, 3), "step_ms_per_8_frames": round(ms_mb, 3),
                                   "frames_per_s": round(N / ms_mb * 1e3, 1),
                                   "mask_share": round(mb_ms * N / mb / ms_mb, 3), "outputs_identical": bool(same)}
    if os.environ.get("SEG_GRAPH", "0") == "1":
        # launch-overhead probe: the mask program (MASK_DT) replayed from a captured HIP graph (static input / output
        # buffers); the captured kernels are the same launches on the same stream
        me_g = deeplab.MaskEngine(model, dev, resolution=256, dtype=MASK_DT)
        static_in = frames.clone()
        me_g.masks(static_in, ids, feather_px=3)  # allocations, plans, resamplers outside the capture
        torch.cuda.synchronize(dev)
        graph = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            me_g.masks(static_in, ids, feather_px=3)
            torch.cuda.synchronize(dev)
            with torch.cuda.graph(graph, stream=s):
                static_out = me_g.masks(static_in, ids, feather_px=3)
        torch.cuda.current_stream(dev).wait_stream(s)
        g_ms = timed(lambda: graph.replay(), STEPS)
        ref = me_g.masks(static_in, ids, feather_px=3)
        graph.replay()
        torch.cuda.synchronize(dev)
        out.update({"mask_ms_graph": round(g_ms, 3), "graph_masks_identical": bool(torch.equal(ref, static_out))})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
