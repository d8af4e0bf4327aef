set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for L in default v1 v2 v3 v4 default; do
  if [ "$L" = default ]; then unset NST_HIP_LIB; else export NST_HIP_LIB=$PWD/sweep/libnst_hip_$L.so; fi
  echo "== $L"
  GATYS_STEPS=100 timeout -k 10 120 python -u tools/gatys_bench.py 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('gatys ms/step', d['ms_per_step'])" || exit 1
done
for L in v1 v2 v3 v4; do
  export NST_HIP_LIB=$PWD/sweep/libnst_hip_$L.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_gatys.py -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -1
done
