#!/bin/bash
# Round-5 closing call: full GPU suite, rocprofv3 kernel-trace + PMC passes (tools/prof_pass.sh), then the bench with
# the fresh PMC summary in place (roofline.traffic / rocprof_* of this build), gather bench, measured peaks.
#   bash tools/gpu_r05r.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05_r}
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v -s --timeout 400 --timeout-method thread \
  > gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo "tests failed rc=$?"; grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_$TAG.log | head -30; tail -20 gpurun_out/gpu_tests_$TAG.log; exit 1; }
grep -E "passed|failed" gpurun_out/gpu_tests_$TAG.log | tail -1
bash tools/prof_pass.sh prof_$TAG || exit 1
cp gpurun_out/prof_$TAG/pmc_res_conv.json profiles/pmc_res_conv.json
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
python tools/bench_brief.py gpurun_out/bench_$TAG.json
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --gather --no-cpu-baseline --no-fp32 --no-fp16 --no-fp32s --no-fp16m > gpurun_out/bench_gather_$TAG.json 2> gpurun_out/bench_gather_$TAG.err || { echo "gather bench failed"; tail -30 gpurun_out/bench_gather_$TAG.err; exit 1; }
timeout -k 10 120 ./tools/peak_bench > gpurun_out/peaks_$TAG.json 2> gpurun_out/peaks_$TAG.err || { echo "peak bench failed"; exit 1; }
cat gpurun_out/peaks_$TAG.json
