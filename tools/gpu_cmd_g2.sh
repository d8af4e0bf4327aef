set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gatys.py tests/test_gpu_deeplab.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_g2.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_g2.log | head -20; tail -30 gpurun_out/gpu_tests_g2.log; exit 1; }
tail -1 gpurun_out/gpu_tests_g2.log
bash tools/gpu_gemm_sweep.sh g2 noglds
