#!/bin/bash
# Round-6 validation of the default build: GPU tests, bench, --gather bench (self-check), the one-rank RCCL process
# group A/B, rocprofv3 kernel trace + PMC passes.   bash tools/gpu_r06f.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r06_f}
bash tools/gpu_all.sh $TAG || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --gather --no-cpu-baseline --no-fp32 --no-fp16 --no-fp16m --no-fp32s \
  > gpurun_out/bench_gather_$TAG.json 2> gpurun_out/bench_gather_$TAG.err || { echo "gather bench failed"; tail -20 gpurun_out/bench_gather_$TAG.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('gather', d['value'], d['gather_verify'])" gpurun_out/bench_gather_$TAG.json
for i in 1 2 3; do
  for pgf in "" "--process-group"; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 $pgf --no-cpu-baseline --no-fp32 --no-fp16 --no-fp16m --no-fp32s \
      > gpurun_out/pg_$TAG.json 2> gpurun_out/pg_$TAG.err || { echo "pg bench failed"; tail -20 gpurun_out/pg_$TAG.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('pg' if sys.argv[2] else 'nopg', d['value'], d['ms_per_step'])" gpurun_out/pg_$TAG.json "$pgf"
  done
done | tee gpurun_out/pg_ab_$TAG.txt
bash tools/prof_pass.sh prof_$TAG && grep -A1 "wst16_kernel<bf16, 8, [02], false, false>" gpurun_out/prof_$TAG/summary.txt
