set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_layers.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_i1.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_i1.log | head -20; tail -30 gpurun_out/gpu_tests_i1.log; exit 1; }
tail -1 gpurun_out/gpu_tests_i1.log
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_i1 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-fp32 --no-fp16 --no-fp32s > gpurun_out/prof_i1.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/prof_i1.log; exit 1; }
grep -h "in_stats\|in_partial\|in_finalize" gpurun_out/prof_i1/run_kernel_stats.csv | cut -d, -f1-5
