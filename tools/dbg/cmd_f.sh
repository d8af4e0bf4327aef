set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_regions.py -m gpu -v --timeout 400 --timeout-method thread -s > gpurun_out/gpu_tests_r04f.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/gpu_tests_r04f.log | head -20; tail -5 gpurun_out/gpu_tests_r04f.log; }
tail -2 gpurun_out/gpu_tests_r04f.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_r04f.json 2> gpurun_out/bench_r04f.err || { echo "bench failed"; tail -30 gpurun_out/bench_r04f.err; exit 1; }
python tools/bench_brief.py gpurun_out/bench_r04f.json
