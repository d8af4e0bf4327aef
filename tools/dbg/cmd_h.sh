set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>: stop the script after a hang / abort / segfault
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?
  echo "== $name rc=$rc"; tail -3 gpurun_out/$name.log
  case $rc in 124|137|134|139) exit 1;; esac
  return 0
}
step h_tests 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_flow.py -m gpu -x -q --timeout 300 --timeout-method thread
NST_PIPE_PROF=1 step h_cli 500 python -u tools/cli_bench.py --frames 240
grep -E "pipe-prof|frames_per_s" gpurun_out/h_cli.log
step h_seg 300 python -u tools/seg_bench.py
