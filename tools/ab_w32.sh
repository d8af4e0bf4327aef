#!/bin/bash
# A/B of the trunk kernels on the bf16 1080p step (tools/batch_sweep.py 8), alternating: NST_WST32=0 (16x16x32
# conv_wstat.hip) vs the default (32x32x16 conv_wst32.hip).   bash tools/ab_w32.sh [rounds]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
for i in $(seq 1 ${1:-2}); do
  for v in 0 1; do
    echo "== NST_WST32=$v"
    NST_WST32=$v timeout -k 10 120 python -u tools/batch_sweep.py 8 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
