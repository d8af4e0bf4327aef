#!/bin/bash
# Round-5 call: parity + per-layer suites, then A/B of library variants over three mode profiles.
#   bash tools/gpu_r05t.sh <tag> <variants...>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
[ -n "$SKIP_TESTS" ] || timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layers.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_$TAG.log | head -20; tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -1 gpurun_out/gpu_tests_$TAG.log
for r in 1 2; do
  for args in "bf16 johnson" "fp32s johnson" "bf16 reconet"; do
    for v in default "$@"; do
      if [ "$v" = default ]; then unset NST_HIP_LIB; else export NST_HIP_LIB="sweep/libnst_hip_$v.so"; fi
      f=gpurun_out/ab_${TAG}_${v}_${args// /_}_$r.json
      timeout -k 10 200 python -u tools/mode_profile.py $args > $f 2> $f.err || { echo "variant $v failed"; tail -5 $f.err; exit 1; }
      python3 tools/ab_line.py "$v $args" $f
    done
  done
done
