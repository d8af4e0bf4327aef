#!/bin/bash
# Layer checks + batch-8 A/B of an experiment library against the default one:
#   bash tools/gpu_ab_lib.sh <lib tag> [pytest -k expression]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/neuralstyletransferv1_amd/libnst_hip_$1.so
K=${2:-"bf16_layers_1080p or (trunk_vs_generic and johnson)"}
NST_HIP_LIB=$L timeout -k 10 400 python -u -m pytest tests/test_gpu_layers.py tests/test_gpu_parity.py -m gpu -x -q -k "$K" \
  --timeout 300 --timeout-method thread > gpurun_out/ab_tests_$1.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/ab_tests_$1.log; exit 1; }
tail -n 1 gpurun_out/ab_tests_$1.log
for i in 1 2; do
  echo "== default"; timeout -k 10 120 python -u tools/batch_sweep.py 8 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== $1"; NST_HIP_LIB=$L timeout -k 10 120 python -u tools/batch_sweep.py 8 2>&1 | grep -v amdgpu.ids || exit 1
done
