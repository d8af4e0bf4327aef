set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
: > gpurun_out/m_sweep.txt
run() {
  env "$@" GATYS_STEPS=200 timeout -k 10 120 python -u tools/gatys_bench.py > gpurun_out/m_one.log 2>&1; rc=$?
  echo "$* rc=$rc $(tail -1 gpurun_out/m_one.log | cut -c100-200)" | tee -a gpurun_out/m_sweep.txt
  [ $rc -eq 0 ] || exit 1
}
run X=0
run NST_GEMM_RING32=4
run NST_VGG_GEMM_B=0x1ffe
run NST_VGG_GEMM_B=0x1ffe NST_GEMM_RING32=4
run NST_GEMM_PF2=0
run X=0
