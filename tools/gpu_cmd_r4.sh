set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for L in default c1a c1b d2a d2b c3a d1a d1b default; do
  if [ "$L" = default ]; then unset NST_HIP_LIB; else export NST_HIP_LIB=$PWD/sweep/libnst_hip_$L.so; fi
  echo "== $L"
  timeout -k 10 120 python -u tools/mode_profile.py bf16 reconet 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['per_layer_ms']; print(d['frames_per_s'], d['ms_per_step'], [p[k] for k in p if k.startswith('encoder.layers.0') or k.startswith('encoder.layers.1') or k.startswith('encoder.layers.2') or k.startswith('decoder')])" || exit 1
done
