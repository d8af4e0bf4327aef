#!/bin/bash
# Kernel-trace + PMC passes of a short bench run on the GPU box (one rocprofv3 run per pass, each
# under its own time limit; counters per pass within the gfx950 slot limits of MI355X_MICROARCH.md).
#   bash tools/prof_pass.sh <tag> [bench args...]
# writes gpurun_out/<tag>/{stats,sq1,sq2,fetch,write}/...csv
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp
TAG=$1; shift
ARGS=${*:---steps 3 --warmup 1 --no-cpu-baseline --no-fp32}
O=gpurun_out/$TAG
mkdir -p "$O"
run() {  # name, then rocprofv3 options
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 "$@" --output-format csv -d "$O/$name" -o run -- python3 bench.py $ARGS \
    > "$O/$name.log" 2>&1 || { echo "pass $name failed rc=$?"; tail -20 "$O/$name.log"; return 1; }
  echo "pass $name ok"
}
run stats --kernel-trace --stats &&
run sq1 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE &&
run sq2 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR &&
run fetch --pmc FETCH_SIZE &&
run write --pmc WRITE_SIZE &&
python3 tools/pmc_summary.py "$O" --json "$O/pmc.json" --res-json "$O/pmc_res_conv.json" > "$O/summary.txt" &&
echo "summary ok"
