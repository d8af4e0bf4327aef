#!/bin/bash
# Round-5 call: fp32s tests (incl. the uint8 first-layer fold) + fp32s / fp16m mode profiles.   bash tools/gpu_r05g.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05_g}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_pipeline_golden.py tests/test_gpu_layers.py -m gpu -x -q -k "fp32s or fold or fp16m" --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_$TAG.log | head -20; tail -20 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$TAG.log
grep -E "fp32s: raw rel|1080p fp32s" gpurun_out/gpu_tests_$TAG.log || true
for dt in fp32s fp16m; do
  timeout -k 10 200 python -u tools/mode_profile.py $dt johnson > gpurun_out/mode_${dt}_$TAG.json 2> gpurun_out/mode_${dt}_$TAG.err || { echo "mode profile $dt failed"; tail -10 gpurun_out/mode_${dt}_$TAG.err; exit 1; }
  cut -c1-400 gpurun_out/mode_${dt}_$TAG.json
done
