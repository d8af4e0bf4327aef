set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_UNALIGNED_STALL SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_u1 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_u1.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/pmc_u1.log; exit 1; }
GATYS_STEPS=5 timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_UNALIGNED_STALL SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_u2 -o run -- python3 tools/gatys_bench.py > gpurun_out/pmc_u2.log 2>&1 || { echo "pmc2 failed"; tail -5 gpurun_out/pmc_u2.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc SQ_LDS_UNALIGNED_STALL SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_u3 -o run -- python3 tools/seg_bench.py > gpurun_out/pmc_u3.log 2>&1 || { echo "pmc3 failed"; tail -5 gpurun_out/pmc_u3.log; exit 1; }
echo done
