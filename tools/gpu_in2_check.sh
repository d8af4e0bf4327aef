#!/bin/bash
# two-stage IN finalize rework: GPU tests, then the IN kernels' times in a kernel trace of a short bench run
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-in2}
bash tools/gpu_all.sh $TAG || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fp32 --no-fp16 --no-fp16m --no-fp32s > gpurun_out/${TAG}_prof.log 2>&1 || { tail -5 gpurun_out/${TAG}_prof.log; exit 1; }
f=$(find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" | head -1)
grep -E "in_stats|in_partial|in_finalize" "$f" | cut -c1-40,100-220
