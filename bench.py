#!/usr/bin/env python3
"""Stylized 1080p frames/s on MI355X (BASELINE.json metric; workload = configs[1]).

One step = one batch of 8 synthetic 1920x1080 uint8 RGB frames per GPU, already resident in
HBM, through the whole hot path on libnst_hip: io_preset encode (imagenet_255, the 'auto'
preset for transformer models) -> Johnson TransformerNet forward (bf16 MFMA, fp32 accumulate;
seeded synthetic checkpoint with the reference's architecture) -> decode + clamp(0,1) +
ToPILImage truncation -> uint8 frames in HBM.

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

Frames shard round-robin across ranks (each rank its own batch, no data-path collective:
scaling "weak"); timing = barrier + synchronize around exactly K steps, max over ranks.
Rank 0 prints ONE JSON line.  Also reported: the dominant kernel's roofline (residual-trunk
3x3 conv, timed live with HIP events on the forward's stream), the reference CPU path timed
on this host (oracle/nst_oracle.py = the reference's own PyTorch-CPU fp32 arithmetic, pinned
bit-exact to golden vectors of the reference modules), and SSIM of the GPU output vs it.
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

H, W, BATCH = 1080, 1920, 8
PRESET = "imagenet_255"
MFMA_BF16_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 (MI355X_MICROARCH.md chip table)
HBM_PEAK_GBS = 8000.0
# Algorithmic work: 307,584 FLOP per output pixel = 637.81 GFLOP per 1080p frame.
FLOP_PER_PIXEL = 307584
# dominant kernel: the 10 residual-trunk convs (3x3, 128->128 at H/4 x W/4): 60% of the FLOPs
RES_FLOP_PER_LAUNCH = 2 * 128 * 128 * 9 * (H // 4) * (W // 4) * BATCH
RES_BYTES_PER_LAUNCH = ((H // 4) * (W // 4) * 128 * 2 * 2) * BATCH  # bf16 activation in + out


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-frames", type=int, default=2, help="1080p frames timed for the CPU baseline")
    return ap.parse_args()


def cpu_baseline(frames_u8: np.ndarray, sd, nframes: int):
    """The reference's per-frame path on this host's cores (oracle = its PyTorch-CPU fp32 math)."""
    from oracle import nst_oracle as O
    threads = torch.get_num_threads()
    O.stylize_u8("johnson", sd, frames_u8[:1, :256, :256], PRESET)  # warm-up (small)
    outs = []
    t0 = time.perf_counter()
    for i in range(nframes):
        outs.append(O.stylize_u8("johnson", sd, frames_u8[i:i + 1], PRESET)[0])
    dt = time.perf_counter() - t0
    return {
        "value": nframes / dt, "unit": "frames/s", "cores": threads, "kind": "port",
        "sample": f"{nframes} synthetic 1920x1080 frames, preset {PRESET} -> Johnson fwd fp32 -> decode/clamp/"
                  f"ToPILImage, torch CPU {threads} threads (os.cpu_count={os.cpu_count()})",
        "s_per_frame": dt / nframes,
    }, outs


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)

    from neuralstyletransferv1_amd import synthetic
    from neuralstyletransferv1_amd.transformer_net import TransformerNet

    sd = synthetic.make_state_dict("johnson", seed=0)
    net = TransformerNet()
    net.load_state_dict(sd)
    net = net.to(dev).eval()
    net.compute_dtype = "bf16"
    eng = net.engine(dev)

    # round-robin shard: rank r owns frames r, r+N, ... (distinct seeded content per rank)
    frames_np = synthetic.make_frames(BATCH, H, W, seed=1000 + rank)
    frames = torch.from_numpy(frames_np).to(dev)
    out = torch.empty_like(frames)

    def step():
        return eng.stylize_u8(frames, PRESET)

    for _ in range(args.warmup):
        out = step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    eng.profile_begin()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    prof = eng.profile_end()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    total_frames = BATCH * args.steps * world
    fps = total_frames / elapsed
    # dominant kernel: the residual-trunk conv without a fused join (conv_wstat.hip, WF_NORM):
    # res1.conv1 and every res*.conv2, 6 launches per step; res2..5.conv1 also join the residual
    # stream in their fill (reported separately in whole_path)
    def _plain(n):  # "res1.conv1.conv2d", "res3.conv2.conv2d", ...
        parts = n.split(".")
        return parts[0] == "res1" or parts[1] == "conv2"
    plain = [(n, ms, c) for (n, ms, c) in prof if n.startswith("res") and _plain(n)]
    joined = [(n, ms, c) for (n, ms, c) in prof if n.startswith("res") and not _plain(n)]
    res_ms = sum(ms for _, ms, _ in plain)
    res_launches = sum(c for _, _, c in plain)
    res_avg_ms = res_ms / max(res_launches, 1)
    joined_avg_ms = sum(ms for _, ms, _ in joined) / max(sum(c for _, _, c in joined), 1)
    achieved_tflops = RES_FLOP_PER_LAUNCH / (res_avg_ms * 1e-3) / 1e12 if res_launches else None
    layer_ms = {n: round(ms / max(c, 1), 4) for (n, ms, c) in prof}
    conv_ms_per_step = sum(ms for _, ms, _ in prof) / args.steps

    traffic = None
    pmc_path = os.path.join(REPO, "profiles", "pmc_res_conv.json")
    if os.path.exists(pmc_path):
        try:
            with open(pmc_path) as f:
                traffic = json.load(f).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

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
        "data": "synthetic (seeded 1920x1080 RGB frames; seeded synthetic Johnson checkpoint with the reference "
                "architecture: the .pth weights are not shipped)",
        "config": {
            "workload": "configs[1]: TransformerNet (Johnson) forward, 1920x1080, batch 8 per GPU, bf16 MFMA / fp32 "
                        "accumulate, io_preset imagenet_255, uint8 frames in/out resident in HBM",
            "global_batch": BATCH * world,
            "frame_hw": [H, W],
            "parallelism": f"frames round-robin over {world} GPU(s), no data-path collective",
        },
        "roofline": {
            "bound": "mfma",
            "kernel": "wstat_kernel<8, WF_NORM> (residual-trunk conv 3x3 128->128 @270x480x8, 6 launches/step)",
            "achieved": round(achieved_tflops, 2) if achieved_tflops else None,
            "peak": MFMA_BF16_PEAK_TFLOPS,
            "unit": "TFLOP/s",
            "frac": round(achieved_tflops / MFMA_BF16_PEAK_TFLOPS, 4) if achieved_tflops else None,
            "traffic": traffic,
            "avg_launch_ms": round(res_avg_ms, 4),
            "flop_per_launch": RES_FLOP_PER_LAUNCH,
            "algorithmic_bytes_per_launch": RES_BYTES_PER_LAUNCH,
        },
        "whole_path": {
            "gflop_per_frame": FLOP_PER_PIXEL * H * W / 1e9,
            "achieved_tflops": round(fps / world * FLOP_PER_PIXEL * H * W / 1e12, 2),
            "frac_of_mfma_peak": round(fps / world * FLOP_PER_PIXEL * H * W / 1e12 / MFMA_BF16_PEAK_TFLOPS, 4),
            "conv_kernel_ms_per_step": round(conv_ms_per_step, 3),
            "trunk_joined_avg_ms": round(joined_avg_ms, 4),
            "per_layer_avg_ms": layer_ms,
        },
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb, cpu_outs = cpu_baseline(frames_np, sd, args.cpu_frames)
        result["cpu_baseline"] = cb
        from oracle import nst_oracle as O
        gpu = out.cpu().numpy()
        ss = [O.ssim(gpu[i], cpu_outs[i]) for i in range(len(cpu_outs))]
        diff = [int(np.abs(gpu[i].astype(int) - cpu_outs[i].astype(int)).max()) for i in range(len(cpu_outs))]
        result["ssim_vs_cpu"] = round(float(min(ss)), 5)
        result["max_abs_lsb_vs_cpu"] = max(diff)
        result["speedup_vs_cpu"] = round(fps / cb["value"], 1)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
