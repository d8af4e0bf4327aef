set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for L in default t1616 t832 default; do
  if [ "$L" = default ]; then unset NST_HIP_LIB; else export NST_HIP_LIB=$PWD/sweep/libnst_hip_$L.so; fi
  echo "== $L"
  timeout -k 10 120 python -u tools/mode_profile.py bf16 reconet 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['per_layer_ms']; print(d['frames_per_s'], d['ms_per_step'], [v for k,v in p.items() if 'encoder.layers.3' in k or 'encoder.layers.4' in k])" || exit 1
done
for L in t1616 t832; do
  export NST_HIP_LIB=$PWD/sweep/libnst_hip_$L.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layers.py -m gpu -x -q -k "reconet" --timeout 300 --timeout-method thread 2>&1 | tail -1
done
