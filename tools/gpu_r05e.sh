#!/bin/bash
# Round-5 call: the split-fp16 output conv (fp32s tests + mode profile), architecture timings, then the rocprofv3
# kernel-trace + PMC passes of the bench (tools/prof_pass.sh).   bash tools/gpu_r05e.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05_e}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_pipeline_golden.py -m gpu -x -q -k "fp32s" --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_$TAG.log | head -20; tail -20 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$TAG.log
for dt in fp32s fp32 fp16m; do
  timeout -k 10 200 python -u tools/mode_profile.py $dt johnson > gpurun_out/mode_${dt}_$TAG.json 2> gpurun_out/mode_${dt}_$TAG.err || { echo "mode profile $dt failed"; tail -10 gpurun_out/mode_${dt}_$TAG.err; exit 1; }
  cut -c1-400 gpurun_out/mode_${dt}_$TAG.json
done
timeout -k 10 200 python -u tools/mode_profile.py bf16 reconet > gpurun_out/mode_reconet_$TAG.json 2>&1 || { echo "reconet profile failed"; exit 1; }
cut -c1-1500 gpurun_out/mode_reconet_$TAG.json
timeout -k 10 300 python -u tools/arch_bench.py > gpurun_out/arch_$TAG.txt 2>&1 || { echo "arch bench failed"; tail -10 gpurun_out/arch_$TAG.txt; exit 1; }
grep frames gpurun_out/arch_$TAG.txt
SEG_DTYPES=fp32s timeout -k 10 300 python -u tools/seg_bench.py > gpurun_out/seg_$TAG.json 2> gpurun_out/seg_$TAG.err || { echo "seg bench failed"; tail -20 gpurun_out/seg_$TAG.err; exit 1; }
cat gpurun_out/seg_$TAG.json
timeout -k 10 400 python -u tools/cli_bench.py --frames 240 --paths frames_dir > gpurun_out/cli_$TAG.txt 2>&1 || { echo "cli bench failed"; tail -20 gpurun_out/cli_$TAG.txt; exit 1; }
tail -1 gpurun_out/cli_$TAG.txt
if [ -n "$PROF" ]; then bash tools/prof_pass.sh prof_$TAG && tail -3 gpurun_out/prof_$TAG/summary.txt; fi
