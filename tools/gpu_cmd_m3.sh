set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_gatys.py tests/test_gpu_deeplab.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_m3.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_m3.log | head -20; tail -30 gpurun_out/gpu_tests_m3.log; exit 1; }
tail -1 gpurun_out/gpu_tests_m3.log
bash tools/gpu_gemm_sweep.sh gemm s0 default s0
GATYS_STEPS=30 timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gatys_m3 -o gatys -- python3 tools/gatys_bench.py > gpurun_out/prof_gatys_m3.log 2>&1 || { echo "gatys prof failed"; tail -20 gpurun_out/prof_gatys_m3.log; exit 1; }
