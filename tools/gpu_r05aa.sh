#!/bin/bash
# Round-5 call: ReCoNet tests, then the mode profile against a kernel-selection flag, two alternating rounds.
#   bash tools/gpu_r05aa.sh <tag> <ksel flag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; K=$2
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layers.py -m gpu -x -q -s -k "reconet" --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_$TAG.log | head -20; tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
grep -E "passed|failed" gpurun_out/gpu_tests_$TAG.log | tail -1
grep -E "frames identical" gpurun_out/gpu_tests_$TAG.log | grep -c True
for r in 1 2; do
  for k in "" $K; do
    MODE_KSEL=$k timeout -k 10 200 python -u tools/mode_profile.py bf16 reconet > gpurun_out/ab_${TAG}_${k:-default}_$r.json 2> gpurun_out/ab_${TAG}_$r.err || { echo "profile failed"; tail -5 gpurun_out/ab_${TAG}_$r.err; exit 1; }
    python3 tools/ab_line.py "${k:-default}" gpurun_out/ab_${TAG}_${k:-default}_$r.json
  done
done
