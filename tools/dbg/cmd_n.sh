set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>: stop the script after a hang / abort / segfault
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?
  echo "== $name rc=$rc"; tail -3 gpurun_out/$name.log | cut -c1-400
  case $rc in 124|137|134|139) exit 1;; esac
  return 0
}
step n_tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layers.py -m gpu -q -s --timeout 300 --timeout-method thread -k "fp16m"
grep -E "1080p x8" gpurun_out/n_tests.log
step n_bench 400 python -u bench.py --steps 20 --warmup 5
python tools/bench_brief.py gpurun_out/n_bench.log | grep -E "fps|fp16m"
step n_reconet 200 python -u tools/mode_profile.py bf16 reconet
for v in t42 t24 t41; do NST_HIP_LIB=sweep/libnst_hip_$v.so step n_reconet_$v 200 python -u tools/mode_profile.py bf16 reconet; done
