#!/bin/bash
# Round-3 check: fp16 per-op debug of ReCoNet(frn), the split-fp16 / Gatys / DeepLab / flow GPU tests, the
# Gatys step timing and the bench (with the fp32s mode).  Each GPU step under its own time limit; a
# crash / timeout (rc > 1) ends the script.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r03d}
timeout -k 10 300 python -u tools/dbg_f16.py reconet_frn tests/golden/model_reconet_frn_s1_48x84.npz > gpurun_out/dbg_frn.txt 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layers.py tests/test_gpu_gatys.py tests/test_gpu_deeplab.py tests/test_gpu_flow.py \
  -m gpu -v -s -k "fp32s or gatys or deeplab or flow or dis or area or reconet" --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/gpu_tests_$T.log | head -20; tail -2 gpurun_out/gpu_tests_$T.log
[ $rc -le 1 ] || { echo "pytest aborted rc=$rc"; exit 1; }
GATYS_STEPS=100 timeout -k 10 300 python -u tools/gatys_bench.py > gpurun_out/gatys_$T.json 2>&1 || { tail -20 gpurun_out/gatys_$T.json; exit 1; }
cat gpurun_out/gatys_$T.json
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || { tail -30 gpurun_out/bench_$T.err; exit 1; }
python tools/bench_brief.py gpurun_out/bench_$T.json
timeout -k 10 300 python -u tools/arch_bench.py > gpurun_out/arch_$T.txt 2>&1 || { tail -20 gpurun_out/arch_$T.txt; exit 1; }
cat gpurun_out/arch_$T.txt
exit $rc
