#!/bin/bash
# One GPU call: parity tests, bench, Gatys bench, post-chain bench, rocprofv3 kernel trace + PMC passes.
#   bash tools/gpu_round.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
TAG=${1:-r02}
bash tools/gpu_all.sh $TAG || exit 1
timeout -k 10 200 python -u tools/gatys_bench.py > gpurun_out/gatys_$TAG.json 2> gpurun_out/gatys_$TAG.err || { echo "gatys bench failed"; tail -5 gpurun_out/gatys_$TAG.err; exit 1; }
cat gpurun_out/gatys_$TAG.json
timeout -k 10 200 python -u tools/post_bench.py > gpurun_out/post_$TAG.txt 2>&1 || { echo "post bench failed"; exit 1; }
cat gpurun_out/post_$TAG.txt | grep -v amdgpu.ids
bash tools/prof_pass.sh prof_$TAG && tail -3 gpurun_out/prof_$TAG/summary.txt
