#!/bin/bash
# A/B of the K-streaming GEMM conv launch shapes (tools/build_variants.sh builds): Gatys 512^2 step and the
# configs[4] DeepLab mask per library build, all in one call (box-to-box spread cancels).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-gemm}
shift
for L in default "$@" default; do
  if [ "$L" = default ]; then unset NST_HIP_LIB; else export NST_HIP_LIB=$PWD/sweep/libnst_hip_$L.so; fi
  echo "== $L"
  GATYS_STEPS=100 timeout -k 10 120 python -u tools/gatys_bench.py 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('gatys ms/step', d['ms_per_step'], 'TF', d['achieved_tflops'])" || exit 1
  timeout -k 10 200 python -u tools/seg_bench.py 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('seg mask bf16', d['mask_ms_bf16'], 'fp16', d['mask_ms_fp16'], 'fp32', d['mask_ms_fp32'], 'fullres TF', d['deeplab_fullres_tflops'])" || exit 1
done
