set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>: stop the script after a hang / abort / segfault
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?
  echo "== $name rc=$rc"; tail -3 gpurun_out/$name.log
  case $rc in 124|137|134|139) exit 1;; esac
  return 0
}
step g_tests 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_regions.py -m gpu -v --timeout 300 --timeout-method thread -s
step g_bench 400 python -u bench.py --steps 20 --warmup 5
python tools/bench_brief.py gpurun_out/g_bench.log
step g_gatys 200 python -u tools/gatys_bench.py
NST_GEMM_T256=1 step g_gatys_t256 200 python -u tools/gatys_bench.py
NST_GEMM_T256=1 step g_t256_tests 300 python -u -m pytest tests/test_gpu_gatys.py tests/test_gpu_deeplab.py -m gpu -x -q --timeout 200 --timeout-method thread
step g_cli 500 python -u tools/cli_bench.py --frames 240
