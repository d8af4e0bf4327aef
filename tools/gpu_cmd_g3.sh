set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
GATYS_STEPS=30 timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gatys_g3 -o gatys -- python3 tools/gatys_bench.py > gpurun_out/prof_gatys_g3.log 2>&1 || { echo "gatys prof failed"; tail -20 gpurun_out/prof_gatys_g3.log; exit 1; }
find gpurun_out/prof_gatys_g3 -name "*kernel_stats*"
