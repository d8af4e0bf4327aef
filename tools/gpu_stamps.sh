#!/bin/bash
# Stamp breakdown + batch-8 timing of trunk-kernel variant libraries (make stamp STAMP_TAG=...), optional layer
# tests on the first one.   TESTS=1 bash tools/gpu_stamps.sh <tag> <lib tag> [<lib tag> ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
if [ -n "$TESTS" ]; then
  NST_HIP_LIB=$PWD/neuralstyletransferv1_amd/libnst_hip_$1.so timeout -k 10 400 python -u -m pytest tests/test_gpu_layers.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/stamp_tests_$TAG.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/stamp_tests_$TAG.log; exit 1; }
  tail -n 1 gpurun_out/stamp_tests_$TAG.log
fi
for L in "$@"; do
  echo "== $L"
  NST_HIP_LIB=$PWD/neuralstyletransferv1_amd/libnst_hip_$L.so timeout -k 10 120 python -u tools/w32_stamps.py 2>&1 | grep -v amdgpu.ids || exit 1
  NST_HIP_LIB=$PWD/neuralstyletransferv1_amd/libnst_hip_$L.so timeout -k 10 120 python -u tools/batch_sweep.py 8 2>&1 | grep -v amdgpu.ids || exit 1
done | tee gpurun_out/stamps_$TAG.txt
