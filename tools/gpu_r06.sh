#!/bin/bash
# Round-6 check of the 32x32x16 trunk kernel (conv_wst32.hip): layer / golden parity, then an A/B against the
# 16x16x32 kernel (NST_WST32=0) on the bf16 1080p step, alternating.   bash tools/gpu_r06.sh <tag> [pytest files]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r06}
SEL=${2:-tests/test_gpu_layers.py tests/test_gpu_parity.py}
timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo "tests failed rc=$?"; grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_$TAG.log | head -30; tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$TAG.log
for i in 1 2; do
  for v in 0 1; do
    echo "== NST_WST32=$v"
    NST_WST32=$v timeout -k 10 120 python -u tools/batch_sweep.py 8 || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ab_$TAG.txt
