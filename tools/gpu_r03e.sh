#!/bin/bash
# Round-3: join diagnostics (fp16 ReCoNet-FRN), re-check of re-calibrated tests, split-fp16 tile sweep
# (per-layer times per library build), rocprofv3 kernel stats of the Gatys step.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r03e
timeout -k 10 600 python -u -m pytest tests/test_gpu_layers.py tests/test_gpu_deeplab.py tests/test_gpu_flow.py -m gpu -v -s \
  -k "fp16-reconet_frn or dis_vs or non_divisor or 16bit_vs_oracle or sky_swap" --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?; grep -E "FAILED|ERROR|differs" gpurun_out/gpu_tests_$T.log | head -20; tail -2 gpurun_out/gpu_tests_$T.log
[ $rc -le 1 ] || { echo "pytest aborted rc=$rc"; exit 1; }
for L in default sweep/libnst_hip_v1.so sweep/libnst_hip_v2.so sweep/libnst_hip_v3.so sweep/libnst_hip_v4.so; do
  if [ "$L" = default ]; then unset NST_HIP_LIB; else export NST_HIP_LIB=$PWD/$L; fi
  timeout -k 10 180 python -u tools/mode_profile.py fp32s >> gpurun_out/sweep_$T.jsonl 2>> gpurun_out/sweep_$T.err || { echo "sweep $L failed"; tail -5 gpurun_out/sweep_$T.err; exit 1; }
done
unset NST_HIP_LIB
cat gpurun_out/sweep_$T.jsonl
GATYS_STEPS=30 timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gatys_$T -o gatys -- python3 tools/gatys_bench.py > gpurun_out/prof_gatys_$T.log 2>&1 || { echo "gatys prof failed"; tail -20 gpurun_out/prof_gatys_$T.log; exit 1; }
find gpurun_out/prof_gatys_$T -name "*stats*" | head
exit $rc
