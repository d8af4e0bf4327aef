#!/bin/bash
# Round-3 GPU check: the named pytest selection (all of its failures reported, no -x), then the bench.
#   bash tools/gpu_r03.sh <tag> [pytest selection...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03}; shift
SEL=${*:-tests}
timeout -k 10 900 python -u -m pytest $SEL -m gpu -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/gpu_tests_$TAG.log | grep -v "^tests.*PASSED" | head -40
tail -3 gpurun_out/gpu_tests_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest aborted rc=$rc"; exit 1; fi
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
python tools/bench_brief.py gpurun_out/bench_$TAG.json
exit $rc
