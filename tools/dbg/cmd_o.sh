set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>: stop the script after a hang / abort / segfault
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?
  echo "== $name rc=$rc"; tail -3 gpurun_out/$name.log | cut -c1-300
  case $rc in 124|137|134|139) exit 1;; esac
  return 0
}
step o_tests 700 python -u -m pytest tests/test_gpu_layers.py tests/test_gpu_parity.py -m gpu -q -s --timeout 300 --timeout-method thread -k "fp16m or reconet"
grep -E "1080p x8|FAILED|passed|failed" gpurun_out/o_tests.log | head
for v in dn24 dn824 up832 up464 c1842 c11632; do NST_HIP_LIB=sweep/libnst_hip_$v.so step o_reconet_$v 200 python -u tools/mode_profile.py bf16 reconet; done
step o_reconet 200 python -u tools/mode_profile.py bf16 reconet
