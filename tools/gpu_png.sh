#!/bin/bash
# GPU PNG writer: its tests, the encoder bench, a rocprofv3 kernel trace of it, the CLI frames_dir PNG path with the
# GPU writer.   bash tools/gpu_png.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-png}
timeout -k 10 300 python -u -m pytest tests/test_gpu_png.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/png_tests_$TAG.log 2>&1 || { echo "png tests failed"; grep -E "FAIL|Error|assert" gpurun_out/png_tests_$TAG.log | head -30; tail -30 gpurun_out/png_tests_$TAG.log; exit 1; }
grep -E "passed|failed|size / raw" gpurun_out/png_tests_$TAG.log | tail -3
timeout -k 10 200 python -u tools/png_bench.py > gpurun_out/png_bench_$TAG.json 2> gpurun_out/png_bench_$TAG.err || { echo "png bench failed"; tail -20 gpurun_out/png_bench_$TAG.err; exit 1; }
cat gpurun_out/png_bench_$TAG.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/png_prof_$TAG -o run -- python3 tools/png_bench.py --reps 5 > gpurun_out/png_prof_$TAG.log 2>&1 || { echo "png prof failed"; tail -20 gpurun_out/png_prof_$TAG.log; exit 1; }
f=$(find gpurun_out/png_prof_$TAG -name "*kernel_stats.csv" | head -1); grep -E "png_" "$f" | cut -c1-160
timeout -k 10 400 python -u tools/cli_bench.py --formats png --paths frames_dir --png_writer gpu > gpurun_out/png_cli_gpu_$TAG.json 2> gpurun_out/png_cli_gpu_$TAG.err || { echo "cli gpu failed"; tail -20 gpurun_out/png_cli_gpu_$TAG.err; exit 1; }
tail -1 gpurun_out/png_cli_gpu_$TAG.json
timeout -k 10 400 python -u tools/cli_bench.py --formats png --paths frames_dir --png_writer fast > gpurun_out/png_cli_fast_$TAG.json 2> gpurun_out/png_cli_fast_$TAG.err || { echo "cli fast failed"; tail -20 gpurun_out/png_cli_fast_$TAG.err; exit 1; }
tail -1 gpurun_out/png_cli_fast_$TAG.json
