#!/bin/bash
# Round-5 A/B of a kernel-selection flag over mode profiles, two alternating rounds.
#   bash tools/gpu_r05ks.sh <tag> <ksel flag> "<dtype arch>" ["<dtype arch>" ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
TAG=$1; K=$2; shift 2
for r in 1 2; do
  for args in "$@"; do
    for k in "" $K; do
      f=gpurun_out/ks_${TAG}_${k:-default}_${args// /_}_$r.json
      MODE_KSEL=$k timeout -k 10 200 python -u tools/mode_profile.py $args > $f 2> $f.err || { echo "profile failed"; tail -5 $f.err; exit 1; }
      python3 tools/ab_line.py "${k:-default} $args" $f
    done
  done
done
