#!/bin/bash
# Round-5 call: ReCoNet tests (goldens, per-layer, kernel A/B) + ReCoNet mode profile + architecture timings.
#   bash tools/gpu_r05h.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05_h}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layers.py -m gpu -x -v -k "reconet" --timeout 300 --timeout-method thread -s > gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_$TAG.log | head -20; tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$TAG.log
grep -E "frames identical" gpurun_out/gpu_tests_$TAG.log || true
for a in reconet reconet_frn; do
  timeout -k 10 200 python -u tools/mode_profile.py bf16 $a > gpurun_out/mode_${a}_$TAG.json 2> gpurun_out/mode_${a}_$TAG.err || { echo "mode profile $a failed"; tail -10 gpurun_out/mode_${a}_$TAG.err; exit 1; }
  cut -c1-1600 gpurun_out/mode_${a}_$TAG.json
done
