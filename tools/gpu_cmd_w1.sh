set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_layers.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_w1.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_w1.log | head -20; tail -30 gpurun_out/gpu_tests_w1.log; exit 1; }
tail -1 gpurun_out/gpu_tests_w1.log
bash tools/abn.sh 2 default w9old
