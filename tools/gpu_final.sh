#!/bin/bash
# Closing validation of a round's tree on the box: every GPU test, smoke(), the default bench and the --gather bench.
#   bash tools/gpu_final.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-final}
bash tools/gpu_all.sh $TAG || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --gather --no-cpu-baseline --no-fp32 --no-fp16 --no-fp16m --no-fp32s \
  > gpurun_out/bench_gather_$TAG.json 2> gpurun_out/bench_gather_$TAG.err || { echo "gather bench failed"; tail -20 gpurun_out/bench_gather_$TAG.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('gather', d['value'], d['gather_verify']['planes_match'], d['gather_verify']['frames_match'])" gpurun_out/bench_gather_$TAG.json
