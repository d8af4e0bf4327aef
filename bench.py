#!/usr/bin/env python3
"""Stylized 1080p frames/s on MI355X (BASELINE.json metric; workload = configs[1]).

One step = one batch of 8 synthetic 1920x1080 uint8 RGB frames per GPU, already resident in
HBM, through the whole hot path on libnst_hip: io_preset encode (imagenet_255, the 'auto'
preset for transformer models) -> Johnson TransformerNet forward (bf16 MFMA, fp32 accumulate;
seeded synthetic checkpoint with the reference's architecture) -> decode + clamp(0,1) +
ToPILImage truncation -> uint8 frames in HBM.

  python bench.py [--gpus N --steps K --warmup W] [--gather] [--frame 3840x2160]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

Frames shard round-robin across ranks (each rank its own batch, no data-path collective:
scaling "weak"); timing = barrier + synchronize around exactly K steps, max over ranks.
--gather adds the video pipeline's exchange to the timed step (configs[3]): every rank's stylized
frames' LAB L planes go to rank 0 in frame order (point-to-point, RCCL over xGMI), rank 0 runs the
LAB lightness EMA (pipeline.py:1942-1978) over all of them in order and returns each smoothed plane
to the frame's owner, which rebuilds RGB, blends 0.9 with the original and D2Hs its own frames.

Rank 0 prints ONE JSON line.  The headline K steps run without instrumentation; a separate
profiled pass (HIP events around every conv launch, on the forward's stream) gives the per-layer
times and the dominant kernel's roofline.  Also reported: the fp32 parity-mode frames/s, and the
reference CPU path (oracle/nst_oracle.py = the reference's PyTorch-CPU fp32 arithmetic, pinned
bit-exact to golden vectors of the reference modules) timed on this host per BASELINE.md §4, with
SSIM / max |d| of the GPU output vs the CPU output.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

BATCH = 8
PRESET = "imagenet_255"
MFMA_BF16_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 (MI355X_MICROARCH.md chip table)
HBM_PEAK_GBS = 8000.0
# measured ceilings beside the spec: back-to-back v_mfma_f32_16x16x32_bf16 on random operands
# at the trunk kernel's occupancy (two waves per SIMD), and a streaming copy, tools/peak_bench.hip
PEAKS_JSON = "profiles/r05_peaks.json"
POWER_JSON = "profiles/r05_at_power.json"
# Algorithmic work: 307,584 FLOP and 822 B (bf16 activations) per output pixel.
FLOP_PER_PIXEL = 307584
BYTES_PER_PIXEL = 822


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frame", type=str, default="1920x1080", help="WxH of the synthetic frames")
    ap.add_argument("--gather", action="store_true",
                    help="time the video pipeline's exchange with the forward (configs[3]): L planes to rank 0, ordered "
                         "LAB EMA there, planes back to the owners, merge + blend + D2H on the owner")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--graph", action=argparse.BooleanOptionalAction, default=True,
                    help="time the step as one HIP-graph replay of the captured forward (engine.capture_u8); "
                         "--no-graph: ~60 eager launches per step (profiles/r06_graph_ab.txt: with a process group "
                         "the eager step runs 1.5 %% slower, the graph step not)")
    ap.add_argument("--no-fp32", action="store_true", help="skip the fp32 parity-mode timing (profiling runs)")
    ap.add_argument("--cpu-frames", type=int, default=3, help="timed 1080p frames per CPU configuration")
    ap.add_argument("--no-fp16", action="store_true", help="skip the fp16-mode timing")
    ap.add_argument("--no-fp32s", action="store_true", help="skip the split-fp16 (fp32s) mode timing")
    ap.add_argument("--no-fp16m", action="store_true", help="skip the split-head fp16 (fp16m) mode timing")
    ap.add_argument("--dist-backend", choices=("nccl", "gloo"), default="nccl",
                    help="process-group backend for --gpus N > 1 (nccl = RCCL over xGMI; gloo stages the exchange "
                         "through host memory, so N ranks can rehearse the multi-GPU command on one GPU)")
    ap.add_argument("--process-group", action="store_true",
                    help="create the process group even for one rank (torch.distributed.run --nproc-per-node 1), so "
                         "the barriers and the max-over-ranks all-reduce run on RCCL with the one GPU a box has")
    ap.add_argument("--device", type=int, default=None,
                    help="GPU index for this rank (default LOCAL_RANK); e.g. 0 to put every rank on one GPU")
    return ap.parse_args()


def _physical_cores() -> int:
    try:
        cores = set()
        with open("/proc/cpuinfo") as f:
            phys = core = None
            for line in f:
                if line.startswith("physical id"):
                    phys = line.split(":")[1].strip()
                elif line.startswith("core id"):
                    core = line.split(":")[1].strip()
                elif not line.strip():
                    if core is not None:
                        cores.add((phys, core))
                    phys = core = None
        return len(cores) or (os.cpu_count() or 1)
    except OSError:
        return os.cpu_count() or 1


def cpu_baseline(frames_u8: np.ndarray, sd, nframes: int):
    """the reference's per-frame path on this host's cores (the oracle = its
    PyTorch-CPU fp32 arithmetic): 1 warm-up frame, then >= 3 timed frames, forward alone (preset ->
    Johnson fwd -> decode/clamp/ToPILImage) and the full chain (+ LAB L-EMA via Pillow/LittleCMS,
    + blend 0.9 with the original: run_videos.py defaults), at all physical cores the process may run
    on (`value`), at this job's CPU share (OMP_NUM_THREADS: 16 cores per GPU on the
    pool) and at 4 threads (pipeline.py:2172 default)."""
    from oracle import nst_oracle as O
    share = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    allc = max(1, min(_physical_cores(), aff))
    prev_threads = torch.get_num_threads()
    runs = {}
    outs = []
    for threads in dict.fromkeys((allc, share, 4)):
        torch.set_num_threads(threads)
        ema = O.LabEMA(True, 0.65)
        O.stylize_u8("johnson", sd, frames_u8[:1], PRESET)  # warm-up frame
        t_fwd = t_post = 0.0
        for i in range(nframes):
            f = frames_u8[i % len(frames_u8)]
            t0 = time.perf_counter()
            u8 = O.stylize_u8("johnson", sd, f[None], PRESET)[0]
            t1 = time.perf_counter()
            sm = ema(u8)
            O.blend_u8(sm, f, None, "keep", 0.9)
            t2 = time.perf_counter()
            t_fwd += t1 - t0
            t_post += t2 - t1
            if threads == share:
                outs.append(u8)
        runs[threads] = {"fwd_s_per_frame": t_fwd / nframes, "chain_s_per_frame": (t_fwd + t_post) / nframes}
    torch.set_num_threads(prev_threads)
    # value = the fastest configuration (the strongest baseline): on a shared GPU host all physical cores can be
    # slower than the job's share (measured r03: 4.98 s/frame at 128 threads vs 2.45 s at 16)
    best = min(runs, key=lambda t: runs[t]["fwd_s_per_frame"])
    main = runs[best]
    return {
        "value": 1.0 / main["fwd_s_per_frame"], "unit": "frames/s", "cores": best, "kind": "port",
        "sample": f"{nframes} timed synthetic 1920x1080 frames after 1 warm-up per configuration; value = forward "
                  f"alone (preset {PRESET} -> Johnson fwd fp32 -> decode/clamp/ToPILImage) at {best} threads, the "
                  f"fastest of {sorted(runs)} ({allc} = all physical cores available to the process)",
        "all_cores_threads": allc,
        "all_cores_frames_per_s": 1.0 / runs[allc]["fwd_s_per_frame"],
        "all_cores_full_chain_frames_per_s": 1.0 / runs[allc]["chain_s_per_frame"],
        "full_chain_frames_per_s": 1.0 / main["chain_s_per_frame"],
        "share_threads": share,
        "share_frames_per_s": 1.0 / runs[share]["fwd_s_per_frame"],
        "share_full_chain_frames_per_s": 1.0 / runs[share]["chain_s_per_frame"],
        "threads4_frames_per_s": 1.0 / runs[4]["fwd_s_per_frame"],
        "threads4_full_chain_frames_per_s": 1.0 / runs[4]["chain_s_per_frame"],
        "s_per_frame": {str(k): v for k, v in runs.items()},
        "host": {"os_cpu_count": os.cpu_count(), "physical_cores": _physical_cores(),
                 "affinity": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None},
    }, outs


def _measured_peaks():
    """The measured MFMA / HBM ceilings kept under profiles/ (mean over its runs), or None."""
    try:
        with open(os.path.join(REPO, PEAKS_JSON)) as f:
            runs = json.load(f)["runs"]
        mf = float(np.mean([r["mfma_bf16_16x16x32_tflops"]["random_2w"] for r in runs]))
        hb = float(np.mean([r["hbm_copy_gbs"] for r in runs]))
        hr = float(np.mean([r.get("hbm_read_gbs", 0.0) for r in runs]))
        return {"mfma_tflops": round(mf, 1), "hbm_copy_gbs": round(hb, 1), "hbm_read_gbs": round(hr, 1),
                "source": PEAKS_JSON,
                "what": "v_mfma_f32_16x16x32_bf16 back to back on random operands at two waves per SIMD; the best "
                        "streaming copy (read + write bytes) and read of tools/peak_bench.hip"}
    except (OSError, KeyError, ValueError):
        return None


def _sustained_power():
    """The step's sustained socket power and compute clocks (profiles/r05_at_power.json, amd-smi beside a long
    back-to-back run of this workload), or None: the MFMA ceiling at the clock the power cap leaves."""
    try:
        with open(os.path.join(REPO, POWER_JSON)) as f:
            d = json.load(f)
        mhz = [v for s in d["samples"] for v in s["gfx_mhz"]]
        w = [s["socket_w"] for s in d["samples"]]
        clk = float(np.mean(mhz)) / d["max_gfx_mhz"]
        return {"socket_w": round(float(np.mean(w)), 1), "board_limit_w": d["board_limit_w"],
                "gfx_mhz": round(float(np.mean(mhz)), 1), "max_gfx_mhz": d["max_gfx_mhz"], "clock_frac": round(clk, 4),
                "mfma_peak_at_clock_tflops": round(MFMA_BF16_PEAK_TFLOPS * clk, 1), "source": POWER_JSON}
    except (OSError, KeyError, ValueError, TypeError):
        return None


def layer_flops(H: int, W: int) -> dict:
    """Algorithmic FLOP per frame of each Johnson layer (transformer_net.py:4-41): 2 cin cout k^2
    per output pixel (the up-convs at the upsampled resolution)."""
    h2, w2, h4, w4 = (H + 1) // 2, (W + 1) // 2, (H + 3) // 4, (W + 3) // 4
    f = {"conv1.conv2d": 2 * 3 * 32 * 81 * H * W, "conv2.conv2d": 2 * 32 * 64 * 9 * h2 * w2,
         "conv3.conv2d": 2 * 64 * 128 * 9 * h4 * w4, "deconv1.conv2d": 2 * 128 * 64 * 9 * h2 * w2,
         "deconv2.conv2d": 2 * 64 * 32 * 9 * H * W, "deconv3.conv2d": 2 * 32 * 3 * 81 * H * W}
    for r in range(1, 6):
        for c in (1, 2):
            f[f"res{r}.conv{c}.conv2d"] = 2 * 128 * 128 * 9 * h4 * w4
    return f


# NST_DT_F16M's split-precision layers and their MFMA issue cost per algorithmic product (nst_api.cpp layer_kdt):
# the first layer 2 fp16 MFMAs (Wh x + Wl x), the down-convs 3 (Wh xh + Wh xl + Wl xh), the first residual block 2
# (Wh xh + Wh xl, conv_ws1s.hip; with NST_KSEL_F16M_TWO_BLOCKS the second block too)
F16M_MFMA_PER_PRODUCT = {"conv1.conv2d": 2, "conv2.conv2d": 3, "conv3.conv2d": 3, "res1.conv1.conv2d": 2,
                         "res1.conv2.conv2d": 2}
# bytes per element each F16M layer reads / writes (fp32 activations in the split head)
F16M_IO_BYTES = {"conv1.conv2d": (2, 4), "conv2.conv2d": (4, 4), "conv3.conv2d": (4, 4), "res1.conv1.conv2d": (4, 4),
                 "res1.conv2.conv2d": (4, 4)}


def _pmc_res() -> dict:
    try:
        with open(os.path.join(REPO, "profiles", "pmc_res_conv.json")) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def mode_roofline(eng, frames, H: int, W: int, nloc: int) -> dict:
    """The dominant kernel of a precision mode (largest share of a profiled step) against the roofline that bounds
    it: its algorithmic FLOP per launch over the fp16 MFMA peak divided by the MFMA issues per product of its
    arithmetic, and its algorithmic HBM bytes per launch over the HBM peak; `bound` is whichever floor is longer,
    and `achieved` / `frac` are in that roofline's unit.  Launch time: HIP events on the forward's stream.  `traffic`
    = the kernel's HBM bytes per launch from the rocprofv3 PMC pass of this kernel build (profiles/pmc_res_conv.json
    `fp16m_conv2`, keyed by the hash of conv_ws2.hip's sources and flags), or None."""
    eng.profile_begin()
    torch.cuda.synchronize(frames.device)
    for _ in range(3):
        eng.stylize_u8(frames, PRESET)
    torch.cuda.synchronize(frames.device)
    prof = eng.profile_end()
    name, ms, cnt = max(prof, key=lambda t: t[1])
    avg_ms = ms / max(cnt, 1)
    fl = layer_flops(H, W)[name] * nloc
    mpp = F16M_MFMA_PER_PRODUCT.get(name, 1)
    mfma_peak = MFMA_BF16_PEAK_TFLOPS / mpp
    tflops = fl / (avg_ms * 1e-3) / 1e12
    cin, cout = {"conv1.conv2d": (3, 32), "conv2.conv2d": (32, 64), "conv3.conv2d": (64, 128),
                 "deconv1.conv2d": (128, 64), "deconv2.conv2d": (64, 32), "deconv3.conv2d": (32, 3)}.get(name, (128, 128))
    ib, ob = F16M_IO_BYTES.get(name, (2, 2))
    stride_in = {"conv2.conv2d": 2, "conv3.conv2d": 2, "deconv1.conv2d": 0.5, "deconv2.conv2d": 0.5}.get(name, 1)
    opix = fl / nloc / (2 * cin * cout * (81 if name in ("conv1.conv2d", "deconv3.conv2d") else 9))
    byts = nloc * opix * (cin * ib * stride_in * stride_in + cout * ob)
    gbs = byts / (avg_ms * 1e-3) / 1e9
    mfma_floor_ms = fl / (mfma_peak * 1e12) * 1e3
    hbm_floor_ms = byts / (HBM_PEAK_GBS * 1e9) * 1e3
    hbm = hbm_floor_ms >= mfma_floor_ms
    traffic, tsrc = None, "no PMC summary for this kernel build"
    pm = _pmc_res().get("fp16m_conv2") if name == "conv2.conv2d" else None
    if pm:
        from neuralstyletransferv1_amd import _lib
        if pm.get("kernel_src_sha16") == _lib.ws2_kernel_sha() and pm.get("hbm_bytes_per_launch"):
            # the PMC pass profiles the bench's 8-frame batch; scale to this launch's frames
            traffic, tsrc = int(pm["hbm_bytes_per_launch"] * nloc / BATCH), f"profiles/pmc_res_conv.json {pm['kernel']}"
        else:
            tsrc = f"PMC summary is of conv_ws2 sources {pm.get('kernel_src_sha16')}, not this build"
    return {"bound": "hbm" if hbm else "mfma", "kernel": name,
            "achieved": round(gbs if hbm else tflops, 2), "peak": HBM_PEAK_GBS if hbm else round(mfma_peak, 1),
            "unit": "GB/s" if hbm else "TFLOP/s", "frac": round((gbs / HBM_PEAK_GBS) if hbm else (tflops / mfma_peak), 4),
            "traffic": traffic, "traffic_source": tsrc, "avg_launch_ms": round(avg_ms, 4),
            "algorithmic_bytes_per_launch": int(byts), "flop_per_launch": fl, "mfma_issues_per_product": mpp,
            "floors_ms": {"mfma": round(mfma_floor_ms, 4), "hbm": round(hbm_floor_ms, 4)},
            "mfma": {"achieved_tflops": round(tflops, 2), "peak_tflops": round(mfma_peak, 1),
                     "frac": round(tflops / mfma_peak, 4)},
            "hbm": {"achieved_gbs": round(gbs, 1), "peak_gbs": HBM_PEAK_GBS, "frac": round(gbs / HBM_PEAK_GBS, 4),
                    "frac_of_measured_copy": (round(gbs / _measured_peaks()["hbm_copy_gbs"], 4)
                                              if _measured_peaks() else None)},
            "per_layer_avg_ms": {n: round(t / max(c, 1), 4) for n, t, c in prof}}


def _kernel_sha() -> str:
    from neuralstyletransferv1_amd import _lib
    return _lib.trunk_kernel_sha()


def main():
    args = parse()
    W, H = (int(v) for v in args.frame.lower().split("x"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    gpu = args.device if args.device is not None else (local if world > 1 else 0)
    pg = world > 1 or args.process_group
    if pg:
        torch.cuda.set_device(gpu)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", gpu)
    torch.cuda.set_device(dev)

    from neuralstyletransferv1_amd import synthetic
    from neuralstyletransferv1_amd.frames import owners, run_pipeline
    from neuralstyletransferv1_amd.postproc import LabSmoother
    from neuralstyletransferv1_amd.transformer_net import TransformerNet

    sd = synthetic.make_state_dict("johnson", seed=0)
    net = TransformerNet()
    net.load_state_dict(sd)
    net = net.to(dev).eval()
    net.compute_dtype = "bf16"
    eng = net.engine(dev)

    # round-robin shard: rank r owns frames r, r+N, ... (distinct seeded content per rank)
    caps = [BATCH] * world
    nloc = caps[rank]
    frames_np = synthetic.make_frames(nloc, H, W, seed=1000 + rank)
    frames = torch.from_numpy(frames_np).to(dev)
    group = list(range(sum(caps)))
    assert sum(1 for o in owners(len(group), world, caps) if o == rank) == nloc
    from neuralstyletransferv1_amd.postproc import blend_frames

    def step():
        return eng.stylize_u8(frames, PRESET)
    if args.graph and not args.gather:
        # the whole forward as one HIP-graph launch per step (engine.capture_u8): the same kernels on the same
        # HBM-resident frames, without the host launching ~60 kernels per step
        from neuralstyletransferv1_amd.engine import capture_u8
        replay, graph_out = capture_u8(eng, frames, PRESET)

        def step():  # noqa: F811
            replay()
            return graph_out

    def run_gather(k):
        """--gather: k groups through the video pipeline's schedule (frames.run_pipeline): each rank stylizes its
        shard, extracts the LAB L plane, rank 0 runs the ordered EMA (alpha 0.65) over the whole group's planes and
        returns each frame's smoothed plane to its owner, which merges it, blends 0.9 with the original and D2Hs
        its own frames into page-locked memory (the per-rank PCIe leg; the encode is host work, tools/cli_bench.py)"""
        ema = LabSmoother(dev, True, 0.65)
        hosts = [torch.empty((nloc, H, W, 3), dtype=torch.uint8, pin_memory=True) for _ in range(2)]
        copy_stream = torch.cuda.Stream(dev)
        done = []

        def stylize(idx):
            out = eng.stylize_u8(frames, PRESET)
            return ema.planes(out), out

        def emit(idx, rows, out):  # as pipeline.py's emit: D2H on a copy stream, the host does not wait here
            fin = blend_frames(ema.merge(out, rows), frames, 0.9)
            copy_stream.wait_stream(torch.cuda.current_stream(dev))
            if len(done) >= 2:
                done[-2].synchronize()  # the page-locked buffer about to be reused has been drained
            with torch.cuda.stream(copy_stream):
                hosts[len(done) % 2].copy_(fin, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(copy_stream)
            fin.record_stream(copy_stream)
            done.append(ev)
        run_pipeline([group] * k, world, rank, stylize, lambda g, full: ema.smooth_planes(full, (H, W)), emit,
                     lambda g: ((1, H * W), torch.uint8), dev, caps)
        for ev in done[-2:]:
            ev.synchronize()

    def verify_gather(k=2):
        """--gather self-check, outside the timed region: k more groups through the same schedule with a fresh EMA
        (the state crosses a group boundary; gather, ordered stage and return leg all run), then rank 0 recomputes
        them single-rank from every rank's regenerated seeded frames and compares the ordered-EMA planes bytewise and
        each owner's final frames (merge + blend 0.9) by their sha256 (gathered from the ranks)."""
        import hashlib
        ema = LabSmoother(dev, True, 0.65)
        got_planes, got_fin = [], []

        def stylize(idx):
            out = eng.stylize_u8(frames, PRESET)
            return ema.planes(out), out

        def root_post(g, full):
            sm = ema.smooth_planes(full, (H, W))
            got_planes.append(sm.clone())
            return sm

        def emit(idx, rows, out):
            got_fin.append(blend_frames(ema.merge(out, rows), frames, 0.9))
        run_pipeline([group] * k, world, rank, stylize, root_post, emit, lambda g: ((1, H * W), torch.uint8), dev, caps)
        torch.cuda.synchronize(dev)

        def sha(ts):
            return hashlib.sha256(b"".join(t.cpu().numpy().tobytes() for t in ts)).hexdigest()[:16]
        shas = [sha(got_fin)]
        if pg:
            shas = [None] * world
            dist.all_gather_object(shas, sha(got_fin))
        if rank != 0:
            return None
        ref = LabSmoother(dev, True, 0.65)
        fr = [torch.from_numpy(synthetic.make_frames(caps[r], H, W, seed=1000 + r)).to(dev) for r in range(world)]
        outs = [eng.stylize_u8(f, PRESET) for f in fr]
        own = owners(len(group), world, caps)
        local = [sum(1 for o in own[:j] if o == own[j]) for j in range(len(group))]  # frame j's index on its owner
        pl = [ref.planes(o) for o in outs]
        planes_ok, fins = True, [[] for _ in range(world)]
        for gi in range(k):
            full = torch.stack([pl[own[j]][local[j]] for j in range(len(group))])
            sm = ref.smooth_planes(full, (H, W))
            planes_ok = planes_ok and gi < len(got_planes) and torch.equal(sm, got_planes[gi])
            for r in range(world):
                rows = torch.stack([sm[j] for j in range(len(group)) if own[j] == r])
                fins[r].append(blend_frames(ref.merge(outs[r], rows), fr[r], 0.9))
        want = [sha(fins[r]) for r in range(world)]
        return {"groups": k, "ranks": world, "planes_match": bool(planes_ok and len(got_planes) == k),
                "frames_match": want == shas, "frames_sha16_per_rank": shas,
                "what": "ordered-EMA planes of every group and each owner's final frames equal a single-rank "
                        "recomputation on rank 0 (every rank's seeded frames regenerated)"}

    # diagnostic only (profiles/r06_pg_ab.txt): NST_BENCH_NO_CLOSING_BARRIER=1 leaves the closing barrier out of
    # the timed region, to separate its cost from the process group's other effects on a one-rank run
    closing_barrier = os.environ.get("NST_BENCH_NO_CLOSING_BARRIER", "0") != "1"

    def timed(k):
        torch.cuda.synchronize(dev)
        if pg:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        out = None
        if args.gather:
            run_gather(k)  # the last group's exchange, EMA, return and D2H belong to the timed work
        else:
            for _ in range(k):
                out = step()
        torch.cuda.synchronize(dev)
        if pg and closing_barrier:
            dist.barrier()
        el = time.perf_counter() - t0
        if pg:
            t = torch.tensor([el], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el, out

    if args.gather:
        run_gather(max(1, args.warmup))
    else:
        for _ in range(args.warmup):
            step()
    elapsed, out = timed(args.steps)           # the headline: no instrumentation
    total_frames = sum(caps) * args.steps
    fps = total_frames / elapsed

    def time_steps(fn, k):
        fn()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / k

    # the GPU side of the reference's default per-frame chain (run_videos.py defaults): forward +
    # LAB lightness EMA (alpha 0.65, frames in order) + uniform blend 0.9 with the original frame
    from neuralstyletransferv1_amd.postproc import blend_frames
    chain_ema = LabSmoother(dev, True, 0.65)

    def chain_step():
        return blend_frames(chain_ema(eng.stylize_u8(frames, PRESET)), frames, 0.9)
    chain_s = time_steps(chain_step, max(3, min(args.steps, 10))) if world == 1 else None
    # the save leg on the GPU (--png_writer gpu, csrc/png_enc.hip): the chain's output as 8 complete PNG files
    png_s, png_ratio = None, None
    if world == 1:
        from neuralstyletransferv1_amd.pngio import encode_png_gpu
        chain_out = chain_step()
        png_s = time_steps(lambda: encode_png_gpu(chain_out), max(3, min(args.steps, 10)))
        _, png_sizes = encode_png_gpu(chain_out)
        png_ratio = float(png_sizes.double().mean().item()) / (H * (W * 3 + 1))

    # the other precision modes, same step: fp16 (NST_DT_F16: the bench kernels with fp16 operands) and
    # split-fp16 (NST_DT_F32S: fp32 activations, fp16 hi/lo operand pairs -- the fp32 parity bars)
    alt_modes = {}
    for key, dt, skip, what in (
            ("fp16_mode", "fp16", args.no_fp16,
             "NST_DT_F16: the bench kernels with fp16 weights/activations (fp16 MFMA, fp32 accumulate)"),
            ("fp16m_mode", "fp16m", args.no_fp16m,
             "NST_DT_F16M: split-fp16 arithmetic (fp32 activations) on the first layer (weights), the down-convs "
             "(operands and weights) and the first residual block (operands), fp16 kernels elsewhere: the +-1 "
             "LSB bar at three quarters of the fp16 rate"),
            ("fp16m_two_blocks_mode", "fp16m:f16m_two_blocks", args.no_fp16m,
             "NST_DT_F16M with NST_KSEL_F16M_TWO_BLOCKS: residual blocks 1 and 2 on the split-operand kernel "
             "(tests/precision_study.py: live max 0.920 LSB instead of 0.958 on the bench frames)"),
            ("fp32s_mode", "fp32s", args.no_fp32s,
             "NST_DT_F32S: fp32 activations, every conv operand an fp16 hi/lo pair (two fp16 MFMAs per K step, "
             "generic kernels): the fp32 parity mode's +-1 LSB bar")):
        if skip or world != 1:
            continue
        dt, _, ks = dt.partition(":")
        net.compute_dtype = dt
        net.kernel_select = frozenset([ks] if ks else [])
        e_alt = net.engine(dev)
        net.compute_dtype = "bf16"
        net.kernel_select = frozenset()
        t_alt = time_steps(lambda: e_alt.stylize_u8(frames, PRESET), max(3, min(args.steps, 10)))
        alt_modes[key] = (e_alt, {"frames_per_s": round(nloc / t_alt, 2), "ms_per_step": round(t_alt * 1e3, 4),
                                  "what": what})
        if dt == "fp16m":
            alt_modes[key][1]["roofline"] = mode_roofline(e_alt, frames, H, W, nloc)

    # profiled pass: per-conv HIP events on the forward's stream
    kp = max(3, min(args.steps, 10))
    measured = _measured_peaks()
    power = _sustained_power()
    eng.profile_begin()
    torch.cuda.synchronize(dev)
    for _ in range(kp):
        eng.stylize_u8(frames, PRESET)
    torch.cuda.synchronize(dev)
    prof = eng.profile_end()

    # dominant kernel: the residual-trunk conv without a fused join (conv_wst16.hip, WF_NORM):
    # res1.conv1 and every res*.conv2, 6 launches per step; res2..5.conv1 also join the residual
    # stream in their fill (reported separately in whole_path)
    def _plain(n):  # "res1.conv1.conv2d", "res3.conv2.conv2d", ...
        parts = n.split(".")
        return parts[0] == "res1" or parts[1] == "conv2"
    hq, wq = (H + 3) // 4, (W + 3) // 4
    res_flop = 2 * 128 * 128 * 9 * hq * wq * nloc
    res_bytes = hq * wq * 128 * 2 * 2 * nloc  # bf16 activation in + out
    plain = [(n, ms, c) for (n, ms, c) in prof if n.startswith("res") and _plain(n)]
    joined = [(n, ms, c) for (n, ms, c) in prof if n.startswith("res") and not _plain(n)]
    res_launches = sum(c for _, _, c in plain)
    res_avg_ms = sum(ms for _, ms, _ in plain) / max(res_launches, 1)
    joined_avg_ms = sum(ms for _, ms, _ in joined) / max(sum(c for _, _, c in joined), 1)
    achieved_tflops = res_flop / (res_avg_ms * 1e-3) / 1e12 if res_launches else None
    layer_ms = {n: round(ms / max(c, 1), 4) for (n, ms, c) in prof}
    conv_ms_per_step = sum(ms for _, ms, _ in prof) / kp

    # HBM traffic of the dominant kernel from the rocprofv3 PMC pass of this same kernel build
    # (tools/prof_pass.sh + tools/pmc_summary.py write it keyed by the hash of the kernel's sources and
    # build flags, _lib.TRUNK_KERNEL_SOURCES); a summary of another version of the kernel is not used
    traffic, traffic_note, prof_us, prof_joined_us = None, "no PMC summary for this kernel build", None, None
    pmc_path = os.path.join(REPO, "profiles", "pmc_res_conv.json")
    if os.path.exists(pmc_path) and (H, W) == (1080, 1920):
        try:
            with open(pmc_path) as f:
                pm = json.load(f)
            if pm.get("kernel_src_sha16") == _kernel_sha():
                traffic, traffic_note = pm.get("hbm_bytes_per_launch"), pm.get("source")
                prof_us = pm.get("avg_us_profiled")
                prof_joined_us = (pm.get("joined") or {}).get("avg_us_profiled")
            else:
                traffic_note = f"PMC summary is of kernel sources {pm.get('kernel_src_sha16')}, not this build"
        except Exception as e:  # noqa: BLE001
            traffic_note = f"unreadable PMC summary: {e}"

    mp = H * W / 1e6
    result = {
        "metric": "stylized 1080p frames/sec at 1/2/4/8 MI355X; SSIM vs CPU ref",
        "value": round(fps, 3),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (seeded RGB frames; seeded synthetic Johnson checkpoint with the reference "
                "architecture: the .pth weights are not shipped)",
        "config": {
            "workload": (f"configs[1]: TransformerNet (Johnson) forward, {W}x{H}, batch {BATCH} per GPU, bf16 MFMA / "
                         f"fp32 accumulate, io_preset {PRESET}, uint8 frames in/out resident in HBM"
                         + ("; + the video pipeline's exchange (configs[3]): L planes to rank 0, ordered LAB EMA, "
                            "smoothed planes back to each frame's owner, merge + blend 0.9 + D2H on the owner"
                            if args.gather else "")),
            "global_batch": sum(caps),
            "frame_hw": [H, W],
            "parallelism": f"frames round-robin over {world} GPU(s), " +
                           ("point-to-point L-plane gather to rank 0 and return to the owners" if args.gather
                            else "no data-path collective"),
            "dist_backend": args.dist_backend if pg else None,
            "ranks_per_gpu": (world if args.device is not None else 1) if world > 1 else 1,
            "step_launch": ("one HIP-graph replay of the captured forward per step" if (args.graph and not args.gather)
                            else "eager kernel launches"),
        },
        "roofline": {
            "bound": "mfma",
            "kernel": (f"wst16_kernel<bf16, 8, WF_NORM> (conv_wst16.hip: residual-trunk conv 3x3 128->128 on 16x16x32 MFMAs, "
                       f"one wave per SIMD, @{hq}x{wq}x{BATCH}, 6 launches/step)"),
            "achieved": round(achieved_tflops, 2) if achieved_tflops else None,
            "peak": MFMA_BF16_PEAK_TFLOPS,
            "unit": "TFLOP/s",
            "frac": round(achieved_tflops / MFMA_BF16_PEAK_TFLOPS, 4) if achieved_tflops else None,
            "traffic": traffic,
            "traffic_source": traffic_note,
            "avg_launch_ms": round(res_avg_ms, 4),
            "flop_per_launch": res_flop,
            "algorithmic_bytes_per_launch": res_bytes,
            "measured_peak": measured,
            "frac_of_measured_peak": (round(achieved_tflops / measured["mfma_tflops"], 4)
                                      if (achieved_tflops and measured) else None),
            # the step holds the board at its power limit: the spec MFMA rate scaled to the sustained clock
            "sustained_power": power,
            "frac_at_sustained_clock": (round(achieved_tflops / power["mfma_peak_at_clock_tflops"], 4)
                                        if (achieved_tflops and power) else None),
            # the same kernel build's rocprofv3 --kernel-trace average (profiles/pmc_res_conv.json; profiled runs
            # clock a few % lower than this un-profiled pass), so the fraction reproduces from the kept summary
            "rocprof_avg_launch_ms": round(prof_us / 1e3, 4) if prof_us else None,
            "rocprof_frac": round(res_flop / (prof_us * 1e-6) / 1e12 / MFMA_BF16_PEAK_TFLOPS, 4) if prof_us else None,
            "joined": {
                "rocprof_avg_launch_ms": round(prof_joined_us / 1e3, 4) if prof_joined_us else None,
                "rocprof_frac": (round(res_flop / (prof_joined_us * 1e-6) / 1e12 / MFMA_BF16_PEAK_TFLOPS, 4)
                                 if prof_joined_us else None),
                "kernel": "wst16_kernel<bf16, 8, WF_RES> (the same conv with the residual join in its fill, 4 launches/step)",
                "avg_launch_ms": round(joined_avg_ms, 4),
                "achieved": round(res_flop / (joined_avg_ms * 1e-3) / 1e12, 2) if joined_avg_ms else None,
                "frac": round(res_flop / (joined_avg_ms * 1e-3) / 1e12 / MFMA_BF16_PEAK_TFLOPS, 4) if joined_avg_ms else None,
                "frac_of_measured_peak": (round(res_flop / (joined_avg_ms * 1e-3) / 1e12 / measured["mfma_tflops"], 4)
                                          if (joined_avg_ms and measured) else None),
                "algorithmic_bytes_per_launch": 2 * res_bytes,
            },
        },
        "whole_path": {
            "gflop_per_frame": FLOP_PER_PIXEL * H * W / 1e9,
            "achieved_tflops": round(fps / world * FLOP_PER_PIXEL * H * W / 1e12, 2),
            "frac_of_mfma_peak": round(fps / world * FLOP_PER_PIXEL * H * W / 1e12 / MFMA_BF16_PEAK_TFLOPS, 4),
            "algorithmic_hbm_gbs": round(fps / world * BYTES_PER_PIXEL * H * W / 1e9, 1),
            "frac_of_hbm_peak": round(fps / world * BYTES_PER_PIXEL * H * W / 1e9 / HBM_PEAK_GBS, 4),
            "profiled_steps": kp,
            "conv_kernel_ms_per_step": round(conv_ms_per_step, 3),
            "trunk_joined_avg_ms": round(joined_avg_ms, 4),
            "per_layer_avg_ms": layer_ms,
            "megapixels_per_frame": mp,
        },
        "cpu_baseline": None,
    }
    if chain_s is not None:
        result["gpu_full_chain"] = {
            "frames_per_s": round(nloc / chain_s, 2),
            "ms_per_step": round(chain_s * 1e3, 4),
            "what": "forward (bf16) + LAB lightness EMA (alpha 0.65, frames in order) + blend 0.9 with the original "
                    "(run_videos.py defaults), one GPU, frames in HBM",
        }
    if png_s is not None:
        result["gpu_png_encode"] = {
            "frames_per_s": round(nloc / png_s, 1), "ms_per_step": round(png_s * 1e3, 4),
            "size_over_raw": round(png_ratio, 4),
            "what": "the chain's output frames as complete PNG files on the GPU (Up filter, per-scanline dynamic-Huffman "
                    "deflate, Adler-32 / CRC-32; csrc/png_enc.hip, --png_writer gpu); lossless"}
    for key, (_, info) in alt_modes.items():
        result[key] = info
    if args.graph and not args.gather:  # the replayed graph's output is the eager forward's, bit for bit
        result["graph_step_matches_eager"] = bool(torch.equal(out, eng.stylize_u8(frames, PRESET)))
    if args.gather:
        vg = verify_gather()
        if rank == 0:
            result["gather_verify"] = vg
    if rank == 0 and world == 1 and not args.no_fp32:
        # the fp32 parity mode (exact-f32 MFMA), same frames
        net.compute_dtype = "fp32"
        e32 = net.engine(dev)
        e32.stylize_u8(frames, PRESET)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(3):
            e32.stylize_u8(frames, PRESET)
        torch.cuda.synchronize(dev)
        result["fp32_parity_frames_per_s"] = round(3 * BATCH / (time.perf_counter() - t0), 2)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and (H, W) == (1080, 1920):
        cb, cpu_outs = cpu_baseline(frames_np, sd, args.cpu_frames)
        result["cpu_baseline"] = cb
        from oracle import nst_oracle as O
        gpu = eng.stylize_u8(frames, PRESET).cpu().numpy()
        k = min(len(cpu_outs), BATCH)
        ss = [O.ssim(gpu[i], cpu_outs[i]) for i in range(k)]
        diff = [np.abs(gpu[i].astype(int) - cpu_outs[i].astype(int)) for i in range(k)]
        result["ssim_vs_cpu"] = round(float(min(ss)), 5)
        result["max_abs_lsb_vs_cpu"] = int(max(d.max() for d in diff))
        result["within_1lsb_vs_cpu"] = round(float(np.mean([(d <= 1).mean() for d in diff])), 6)
        result["within_2lsb_vs_cpu"] = round(float(np.mean([(d <= 2).mean() for d in diff])), 6)
        result["speedup_vs_cpu"] = round(fps / cb["value"], 1)
        for key, (e_alt, info) in alt_modes.items():
            ga = e_alt.stylize_u8(frames, PRESET).cpu().numpy()
            da = [np.abs(ga[i].astype(int) - cpu_outs[i].astype(int)) for i in range(k)]
            info.update({
                "ssim_vs_cpu": round(float(min(O.ssim(ga[i], cpu_outs[i]) for i in range(k))), 6),
                "max_abs_lsb_vs_cpu": int(max(d.max() for d in da)),
                "within_1lsb_values": round(float(np.mean([(d <= 1).mean() for d in da])), 6),
                "within_1lsb_pixels": round(float(np.mean([(d.max(-1) <= 1).mean() for d in da])), 6),
            })
    if rank == 0:
        print(json.dumps(result), flush=True)
    if pg:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
