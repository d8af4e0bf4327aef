#!/bin/bash
# Round-5 A/B: ReCoNet kernel variants (sweep/libnst_hip_*.so), two alternating rounds.   bash tools/gpu_r05i.sh <tag> <variants...>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
TAG=$1; shift
for r in 1 2; do
  for v in default "$@"; do
    if [ "$v" = default ]; then unset NST_HIP_LIB; else export NST_HIP_LIB="sweep/libnst_hip_$v.so"; fi
    timeout -k 10 200 python -u tools/mode_profile.py ${AB_ARGS:-bf16 reconet} > gpurun_out/ab_${TAG}_${v}_$r.json 2> gpurun_out/ab_${TAG}_${v}_$r.err || { echo "variant $v failed"; tail -5 gpurun_out/ab_${TAG}_${v}_$r.err; exit 1; }
    python3 tools/ab_line.py "$v" gpurun_out/ab_${TAG}_${v}_$r.json
  done
done
