set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>: stop the script after a hang / abort / segfault
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?
  echo "== $name rc=$rc"; tail -1 gpurun_out/$name.log | cut -c1-300
  case $rc in 124|137|134|139) exit 1;; esac
  return 0
}
step r2_bench 400 python -u bench.py
python tools/bench_brief.py gpurun_out/r2_bench.log | head -3
bash tools/prof_pass.sh prof_r04_r2 || exit 1
: > gpurun_out/r2_gatys_sweep.txt
for m in "X=0" "NST_VGG_GEMM_F=0x1ff0 NST_VGG_GEMM_B=0x1ff0" "NST_VGG_GEMM_F=0x1f00 NST_VGG_GEMM_B=0x1f00" "NST_VGG_GEMM_B=0x1ff0"; do
  env $m GATYS_STEPS=200 timeout -k 10 120 python -u tools/gatys_bench.py > gpurun_out/r2_one.log 2>&1 || exit 1
  echo "$m $(tail -1 gpurun_out/r2_one.log | cut -c100-160)" | tee -a gpurun_out/r2_gatys_sweep.txt
done
