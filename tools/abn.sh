#!/bin/bash
# A/B/... timing of library builds on one box: bash tools/abn.sh name1 name2 ... (libnst_hip_<name>.so; "base" first)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
for r in 1 2; do
  for n in "$@"; do
    echo "== $n"
    NST_HIP_LIB=$PWD/neuralstyletransferv1_amd/libnst_hip_$n.so timeout -k 10 120 python -u tools/batch_sweep.py 8 2>&1 | grep batch || exit 1
  done
done
