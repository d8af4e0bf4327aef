#!/bin/bash
# Round-5 experiment call: A/B of library variants (tools/abn.sh) and the configs[4] bench with mask batches.
#   bash tools/gpu_r05x.sh <tag> <rounds> <variant>...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; R=$2; shift 2
timeout -k 10 600 bash tools/abn.sh $R default "$@" > gpurun_out/abn_$TAG.txt 2>&1 || { echo "abn failed"; tail -20 gpurun_out/abn_$TAG.txt; exit 1; }
cat gpurun_out/abn_$TAG.txt
if [ -n "$SEG" ]; then
  SEG_DTYPES=fp32s,bf16 timeout -k 10 300 python -u tools/seg_bench.py > gpurun_out/seg_$TAG.json 2> gpurun_out/seg_$TAG.err || { echo "seg bench failed"; tail -20 gpurun_out/seg_$TAG.err; exit 1; }
  cat gpurun_out/seg_$TAG.json
fi
