set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_m5.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_m5.log | head -20; tail -30 gpurun_out/gpu_tests_m5.log; exit 1; }
tail -1 gpurun_out/gpu_tests_m5.log
bash tools/gpu_gemm_sweep.sh gemm prev default prev
