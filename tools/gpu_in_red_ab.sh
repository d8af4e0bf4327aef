#!/bin/bash
# A/B of the two-stage IN reduce's channels per block (NST_IN_RED_CH): kernel times from kernel traces of a short bench
# (profiles/r06_in_red_ab.txt; the NST_IN_RED_CH selector in nst_ops.hip launch_in_finalize was removed after it: re-add to rerun)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-inred}
for ch in 16 8 32 64; do
  NST_IN_RED_CH=$ch timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_$ch -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fp32 --no-fp16 --no-fp16m --no-fp32s > gpurun_out/${TAG}_$ch.log 2>&1 || { echo "prof $ch failed"; tail -5 gpurun_out/${TAG}_$ch.log; exit 1; }
  f=$(find gpurun_out/${TAG}_$ch -name "*kernel_stats.csv" | head -1)
  echo "ch $ch: $(grep in_partial_reduce "$f" | awk -F'",' '{print $2}')"
done | tee gpurun_out/${TAG}_prof.txt
