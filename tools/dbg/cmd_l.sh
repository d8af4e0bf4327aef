set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>: stop the script after a hang / abort / segfault
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?
  echo "== $name rc=$rc"; tail -3 gpurun_out/$name.log | cut -c1-700
  case $rc in 124|137|134|139) exit 1;; esac
  return 0
}
NST_GEMM_GLDS_F32=1 step l_tests 500 python -u -m pytest tests/test_gpu_deeplab.py -m gpu -x -q --timeout 200 --timeout-method thread -k "fp32"
NST_GEMM_GLDS_F32=1 SEG_DTYPES=fp32,fp32s step l_seg_glds 300 python -u tools/seg_bench.py
SEG_DTYPES=fp32,fp32s step l_seg 300 python -u tools/seg_bench.py
