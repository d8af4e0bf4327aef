#!/bin/bash
# A/B timing of two library builds on one box (alternating, same frames): bash tools/ab.sh [libA] [libB] [rounds]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
A=${1:-neuralstyletransferv1_amd/libnst_hip_base.so}
B=${2:-neuralstyletransferv1_amd/libnst_hip.so}
R=${3:-2}
for i in $(seq 1 $R); do
  for L in $A $B; do
    echo "== $L"
    NST_HIP_LIB=$PWD/$L timeout -k 10 120 python -u tools/batch_sweep.py 8 || exit 1
  done
done
