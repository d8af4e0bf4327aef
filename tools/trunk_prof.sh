#!/bin/bash
# rocprofv3 kernel trace + PMC passes of the bf16 1080p step (tools/batch_sweep.py 8), one run per pass, for the
# trunk-kernel A/B (NST_WST32=0: 16x16x32 wstat; 1: 32x32x16 wst32).   bash tools/trunk_prof.sh <tag> [0|1 ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp
TAG=$1; shift
VARS=${*:-0 1}
for v in $VARS; do
  O=gpurun_out/$TAG/w$v
  mkdir -p "$O"
  run() {
    local name=$1; shift
    NST_WST32=$v timeout -s KILL 90 rocprofv3 "$@" --output-format csv -d "$O/$name" -o run -- python3 tools/batch_sweep.py 8 \
      > "$O/$name.log" 2>&1 || { echo "pass $name failed rc=$?"; tail -20 "$O/$name.log"; return 1; }
  }
  run stats --kernel-trace --stats &&
  run sq1 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE &&
  run sq2 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR &&
  run sq3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA &&
  python3 tools/pmc_summary.py "$O" > "$O/summary.txt" && grep -A1 "wst" "$O/summary.txt" || exit 1
done
