#!/bin/bash
# HIP-graph step vs eager launches, with and without a one-rank RCCL process group, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
for i in 1 2 3; do
  for mode in eager graph pg_eager pg_graph; do
    a=""; [ ${mode#pg_} = graph ] && a="--graph"
    [ ${mode%%_*} = pg ] && a="$a --process-group"
    RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29520 + i)) \
      timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 $a --no-cpu-baseline --no-fp32 --no-fp16 --no-fp16m --no-fp32s \
      > gpurun_out/gr.json 2> gpurun_out/gr.err || { echo "bench failed $mode"; tail -8 gpurun_out/gr.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/gr.json $mode
  done
done | tee gpurun_out/graph_ab.txt
