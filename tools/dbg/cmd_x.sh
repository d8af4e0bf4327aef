set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for v in o18 o26 o24; do
  NST_HIP_LIB=sweep/libnst_hip_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_layers.py -m gpu -q -x --timeout 200 --timeout-method thread -k "reconet and not frn and bf16" > gpurun_out/x_t_$v.log 2>&1; echo "$v tests rc=$?"; tail -1 gpurun_out/x_t_$v.log
  NST_HIP_LIB=sweep/libnst_hip_$v.so timeout -k 10 120 python -u tools/mode_profile.py bf16 reconet > gpurun_out/x_p_$v.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/x_p_$v.log').read().strip().splitlines()[-1]);print('$v', d['frames_per_s'], d['per_layer_ms']['decoder.layers.4.layers.0.layers.1'])"
done
timeout -k 10 120 python -u tools/mode_profile.py bf16 reconet > gpurun_out/x_p.log 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/x_p.log').read().strip().splitlines()[-1]);print('default', d['frames_per_s'], d['per_layer_ms']['decoder.layers.4.layers.0.layers.1'])"
