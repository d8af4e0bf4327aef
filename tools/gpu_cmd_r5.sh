set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layers.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r5.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_r5.log | head -20; tail -30 gpurun_out/gpu_tests_r5.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r5.log
timeout -k 10 300 python -u tools/arch_bench.py 2>&1 | grep -v amdgpu.ids
