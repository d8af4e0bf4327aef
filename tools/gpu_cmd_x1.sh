set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for pair in "default fp32s" "xs32s fp32s" "default fp32" "xs32 fp32"; do
  set -- $pair
  if [ "$1" = default ]; then unset NST_HIP_LIB; else export NST_HIP_LIB=$PWD/sweep/libnst_hip_$1.so; fi
  echo "== $1 $2"
  timeout -k 10 180 python -u tools/mode_profile.py $2 johnson 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['per_layer_ms']; print(d['frames_per_s'], d['ms_per_step'], p.get('deconv3.conv2d'))" || exit 1
done
for L in xs32s xs32; do
  export NST_HIP_LIB=$PWD/sweep/libnst_hip_$L.so
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -3
done
