#!/bin/bash
# Round-3 measurement: full GPU parity suite, the bench, then rocprofv3 kernel-trace + PMC passes.
#   bash tools/gpu_r03.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo "tests failed rc=$?"; grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_$TAG.log | head -30; tail -20 gpurun_out/gpu_tests_$TAG.log; exit 1; }
grep -E "passed|failed" gpurun_out/gpu_tests_$TAG.log | tail -2
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
python tools/bench_brief.py gpurun_out/bench_$TAG.json
bash tools/prof_pass.sh prof_$TAG
