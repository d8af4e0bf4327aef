#!/bin/bash
# A/B timing of library builds on one box, alternating (same frames, batch 8 1080p bf16 per-layer profile):
#   bash tools/abn.sh <rounds> <lib> <lib> ...   (lib "default" = neuralstyletransferv1_amd/libnst_hip.so,
#   otherwise sweep/libnst_hip_<name>.so from tools/build_variants.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
R=$1; shift
for i in $(seq 1 $R); do
  for L in "$@"; do
    if [ "$L" = default ]; then unset NST_HIP_LIB; else export NST_HIP_LIB=$PWD/sweep/libnst_hip_$L.so; fi
    echo "== $L"
    timeout -k 10 120 python -u tools/batch_sweep.py 8 2>&1 | grep batch || exit 1
  done
done
