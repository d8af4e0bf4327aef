set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_gatys.py tests/test_gpu_parity.py -k "gatys or gram or vgg" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_g6.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_g6.log | head -20; tail -30 gpurun_out/gpu_tests_g6.log; exit 1; }
tail -1 gpurun_out/gpu_tests_g6.log
for L in default prev default prev default; do
  if [ "$L" = default ]; then unset NST_HIP_LIB; else export NST_HIP_LIB=$PWD/sweep/libnst_hip_$L.so; fi
  GATYS_STEPS=100 timeout -k 10 120 python -u tools/gatys_bench.py 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$L gatys ms/step', d['ms_per_step'], 'loss', repr(d['loss_first']), repr(d['loss_last']))" || exit 1
done
unset NST_HIP_LIB
GATYS_STEPS=30 timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gatys_g6 -o gatys -- python3 tools/gatys_bench.py > gpurun_out/prof_gatys_g6.log 2>&1 || { echo "gatys prof failed"; tail -20 gpurun_out/prof_gatys_g6.log; exit 1; }
