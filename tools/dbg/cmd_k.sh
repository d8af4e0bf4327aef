set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>: stop the script after a hang / abort / segfault
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?
  echo "== $name rc=$rc"; tail -3 gpurun_out/$name.log | cut -c1-600
  case $rc in 124|137|134|139) exit 1;; esac
  return 0
}
step k_tests 500 python -u -m pytest tests/test_gpu_deeplab.py tests/test_gpu_gatys.py -m gpu -x -q --timeout 200 --timeout-method thread
step k_gatys 200 python -u tools/gatys_bench.py
NST_GEMM_T256=1 step k_gatys_t256 200 python -u tools/gatys_bench.py
NST_GEMM_PF2=0 step k_seg_pf1 300 python -u tools/seg_bench.py
step k_seg 300 python -u tools/seg_bench.py
