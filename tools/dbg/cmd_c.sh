set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp

timeout -k 10 1000 python -u -m pytest tests -m gpu -x --deselect tests/test_gpu_asan.py -v --timeout 400 --timeout-method thread -s > gpurun_out/gpu_tests_r04d.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/gpu_tests_r04d.log | head -20; tail -5 gpurun_out/gpu_tests_r04d.log; exit 1; }
tail -2 gpurun_out/gpu_tests_r04d.log
grep -E "1080p x8|fp16m" gpurun_out/gpu_tests_r04d.log | head -20
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_r04d.json 2> gpurun_out/bench_r04d.err || { echo "bench failed"; tail -30 gpurun_out/bench_r04d.err; exit 1; }
python tools/bench_brief.py gpurun_out/bench_r04d.json
