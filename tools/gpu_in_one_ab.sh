#!/bin/bash
# A/B of the one-launch IN statistics kernel's channels per block (NST_IN_ONE_CH 16 / 8 / 4): kernel time from a
# rocprofv3 kernel trace of a short bench run, then the bench step alternating.   bash tools/gpu_in_one_ab.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-inone}
X="--no-cpu-baseline --no-fp32 --no-fp16 --no-fp16m --no-fp32s"
for ch in 4 2; do
  NST_IN_ONE_CH=$ch timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_$ch -o run -- python3 bench.py --steps 5 --warmup 2 $X > gpurun_out/${TAG}_$ch.log 2>&1 || { echo "prof $ch failed"; tail -5 gpurun_out/${TAG}_$ch.log; exit 1; }
  f=$(find gpurun_out/${TAG}_$ch -name "*kernel_stats.csv" | head -1)
  echo "ch $ch: $(grep in_stats_kernel "$f" | awk -F'",' '{print $2}')"
done | tee gpurun_out/${TAG}_prof.txt
for r in 1 2; do
  for ch in 4 2; do
    NST_IN_ONE_CH=$ch timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 $X > gpurun_out/${TAG}_b.json 2> gpurun_out/${TAG}_b.err || { echo "bench failed"; tail -5 gpurun_out/${TAG}_b.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('ch', sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/${TAG}_b.json $ch
  done
done | tee gpurun_out/${TAG}_bench.txt
