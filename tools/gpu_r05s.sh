#!/bin/bash
# Round-5 call: NST_DT_F16M with conv3 on fp16 weights (split operand): its tests, then mode profiles against the
# split-weight conv3 (NST_KSEL_F16M_CONV3_SPLIT_W), two alternating rounds.   bash tools/gpu_r05s.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05_s}
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_pipeline_golden.py tests/test_gpu_layers.py -m gpu -x -v -s -k "fp16m" --timeout 400 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_$TAG.log | head -20; tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
grep -E "passed|failed" gpurun_out/gpu_tests_$TAG.log | tail -1
grep -E "1080p x8 fp16m|NST fp16m" gpurun_out/gpu_tests_$TAG.log || true
for r in 1 2; do
  for k in "" f16m_conv3_split_w; do
    MODE_KSEL=$k timeout -k 10 200 python -u tools/mode_profile.py fp16m johnson > gpurun_out/ab_${TAG}_${k:-default}_$r.json 2> gpurun_out/ab_${TAG}_$r.err || { echo "profile failed"; tail -5 gpurun_out/ab_${TAG}_$r.err; exit 1; }
    python3 tools/ab_line.py "${k:-default}" gpurun_out/ab_${TAG}_${k:-default}_$r.json
  done
done
