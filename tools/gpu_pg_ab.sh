#!/bin/bash
# One-rank RCCL process group: where the ~1.5 % goes.  bench.py without a PG, with it, and with it but without the
# closing barrier in the timed region (NST_BENCH_NO_CLOSING_BARRIER=1, diagnostic), alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
for i in 1 2 3; do
  for mode in nopg pg pg_nobar; do
    pgf=""; nb=0
    [ $mode != nopg ] && pgf="--process-group"
    [ $mode = pg_nobar ] && nb=1
    NST_BENCH_NO_CLOSING_BARRIER=$nb RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29510 + i)) \
      timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 $pgf --no-cpu-baseline --no-fp32 --no-fp16 --no-fp16m --no-fp32s \
      > gpurun_out/pg2.json 2> gpurun_out/pg2.err || { echo "bench failed"; tail -5 gpurun_out/pg2.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['whole_path']['conv_kernel_ms_per_step'])" gpurun_out/pg2.json $mode
  done
done | tee gpurun_out/pg_ab2.txt
