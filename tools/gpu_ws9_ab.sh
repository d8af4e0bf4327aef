#!/bin/bash
# conv_ws9 output-tile swizzle: layer / golden checks on the default library, batch-8 A/B against the former
# swizzle (libnst_hip_ws9old.so), and one LDS-conflict PMC pass of each.   bash tools/gpu_ws9_ab.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-ws9}
timeout -k 10 600 python -u -m pytest tests/test_gpu_layers.py tests/test_gpu_parity.py tests/test_gpu_pipeline.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/tests_$TAG.log; exit 1; }
tail -n 1 gpurun_out/tests_$TAG.log
OLD=$PWD/neuralstyletransferv1_amd/libnst_hip_ws9old.so
for i in 1 2; do
  echo "== new"; timeout -k 10 120 python -u tools/batch_sweep.py 8 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== old"; NST_HIP_LIB=$OLD timeout -k 10 120 python -u tools/batch_sweep.py 8 2>&1 | grep -v amdgpu.ids || exit 1
done | tee gpurun_out/ab_$TAG.txt
for v in new old; do
  if [ $v = old ]; then export NST_HIP_LIB=$OLD; else unset NST_HIP_LIB; fi
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES --output-format csv \
    -d gpurun_out/pmc_$TAG/$v -o run -- python3 tools/batch_sweep.py 8 > gpurun_out/pmc_${TAG}_$v.log 2>&1 || { echo "pmc $v failed"; exit 1; }
  python3 - gpurun_out/pmc_$TAG/$v <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "ws9_kernel" in r["Kernel_Name"]:
            acc[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in acc.items():
    print(sys.argv[1].split("/")[-1], k, "conflict/active %.3f" % (v["SQ_LDS_BANK_CONFLICT"] / max(v["SQ_LDS_IDX_ACTIVE"], 1)))
PY
done
# the one-rank RCCL process group A/B: bench.py with and without --process-group, alternating
for i in 1 2 3; do
  for pgf in "" "--process-group"; do
    RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29500 + i)) timeout -k 10 300 python -u bench.py \
      --steps 20 --warmup 3 $pgf --no-cpu-baseline --no-fp32 --no-fp16 --no-fp16m --no-fp32s > gpurun_out/pg_$TAG.json 2> gpurun_out/pg_$TAG.err \
      || { echo "pg bench failed"; tail -5 gpurun_out/pg_$TAG.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('pg' if sys.argv[2] else 'nopg', d['value'], d['ms_per_step'])" gpurun_out/pg_$TAG.json "$pgf"
  done
done | tee gpurun_out/pg_ab_$TAG.txt
