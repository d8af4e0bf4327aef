set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_regions.py tests/test_gpu_flow.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_c2.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_c2.log | head -20; tail -30 gpurun_out/gpu_tests_c2.log; exit 1; }
tail -1 gpurun_out/gpu_tests_c2.log
timeout -k 10 400 python -u tools/cli_bench.py --frames 48 > gpurun_out/cli_c2.json 2>&1 || { tail -20 gpurun_out/cli_c2.json; exit 1; }
tail -1 gpurun_out/cli_c2.json
