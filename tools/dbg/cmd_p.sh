set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>: stop the script after a hang / abort / segfault
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?
  echo "== $name rc=$rc"; tail -3 gpurun_out/$name.log | cut -c1-300
  case $rc in 124|137|134|139) exit 1;; esac
  return 0
}
step p_tests 900 python -u -m pytest tests/test_gpu_layers.py tests/test_gpu_parity.py tests/test_gpu_pipeline.py -m gpu -q --timeout 300 --timeout-method thread -k "reconet or fp32s or fp32 or frn"
grep -E "FAILED|passed|failed" gpurun_out/p_tests.log | head
for a in reconet reconet_frn; do for d in bf16 fp16; do step p_prof_${a}_$d 200 python -u tools/mode_profile.py $d $a; done; done
step p_prof_johnson_fp32s 200 python -u tools/mode_profile.py fp32s johnson
step p_prof_johnson_fp32 200 python -u tools/mode_profile.py fp32 johnson
for v in up4322 up4162 up8162; do
  NST_HIP_LIB=sweep/libnst_hip_$v.so step q_layers_$v 300 python -u -m pytest tests/test_gpu_layers.py -m gpu -q -x --timeout 200 --timeout-method thread -k "reconet and not frn and bf16"
  NST_HIP_LIB=sweep/libnst_hip_$v.so step q_prof_$v 200 python -u tools/mode_profile.py bf16 reconet
done
