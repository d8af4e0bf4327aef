#!/bin/bash
# Round-5 validation call: GPU suite, bench, gather (1080p, 4K), configs[4] seg bench, CLI bench (1 rank and
# 2 gloo ranks).  Each step under its own limit; stop at the first failure.   bash tools/gpu_r05d.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05_d}
bash tools/gpu_r05.sh $TAG ${SEL:-tests} || exit 1
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --gather --frame 3840x2160 --no-cpu-baseline --no-fp32 --no-fp16 --no-fp32s --no-fp16m > gpurun_out/bench_gather4k_$TAG.json 2> gpurun_out/bench_gather4k_$TAG.err || { echo "4K gather bench failed"; tail -20 gpurun_out/bench_gather4k_$TAG.err; exit 1; }
python tools/bench_brief.py gpurun_out/bench_gather4k_$TAG.json | head -1
SEG_DTYPES=fp32s,bf16 timeout -k 10 300 python -u tools/seg_bench.py > gpurun_out/seg_$TAG.json 2> gpurun_out/seg_$TAG.err || { echo "seg bench failed"; tail -20 gpurun_out/seg_$TAG.err; exit 1; }
cat gpurun_out/seg_$TAG.json
timeout -k 10 400 python -u tools/cli_bench.py --frames 240 > gpurun_out/cli_$TAG.txt 2>&1 || { echo "cli bench failed"; tail -20 gpurun_out/cli_$TAG.txt; exit 1; }
tail -1 gpurun_out/cli_$TAG.txt
timeout -k 10 400 python -u tools/cli_bench.py --frames 240 --gpus 2 --paths frames_dir > gpurun_out/cli2_$TAG.txt 2>&1 || { echo "cli bench (2 ranks) failed"; tail -20 gpurun_out/cli2_$TAG.txt; exit 1; }
tail -1 gpurun_out/cli2_$TAG.txt
