#!/bin/bash
# one GPU test file (default: the pipeline tests) on the box.   bash tools/gpu_pipe_tests.sh <tag> [test path]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pipe}
SEL=${2:-tests/test_gpu_pipeline.py}
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/pipe_tests_$TAG.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/pipe_tests_$TAG.log | head -30; tail -30 gpurun_out/pipe_tests_$TAG.log; exit 1; }
grep -E "passed|failed" gpurun_out/pipe_tests_$TAG.log | tail -2
