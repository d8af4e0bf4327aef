set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_deeplab.py tests/test_gpu_regions.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_d1.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_d1.log | head -20; tail -30 gpurun_out/gpu_tests_d1.log; exit 1; }
tail -1 gpurun_out/gpu_tests_d1.log
bash tools/gpu_gemm_sweep.sh d1 nof32
