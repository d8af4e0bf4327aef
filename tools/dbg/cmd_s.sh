set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
: > gpurun_out/s_gatys_sweep.txt
for m in "X=0" "NST_VGG_GEMM_F=0x1f00 NST_VGG_GEMM_B=0x1f00" "NST_VGG_GEMM_F=0x1000 NST_VGG_GEMM_B=0x1f00" "NST_VGG_GEMM_F=0x1f00 NST_VGG_GEMM_B=0x1e00" "NST_VGG_GEMM_F=0x1f00 NST_VGG_GEMM_B=0x1c00" "NST_VGG_GEMM_F=0x1f00 NST_VGG_GEMM_B=0x1000" "NST_VGG_GEMM_F=0x1000 NST_VGG_GEMM_B=0x1000" "NST_VGG_GEMM_F=0x1f00 NST_VGG_GEMM_B=0x0" "X=0"; do
  env $m GATYS_STEPS=200 timeout -k 10 120 python -u tools/gatys_bench.py > gpurun_out/s_one.log 2>&1 || exit 1
  echo "$m $(tail -1 gpurun_out/s_one.log | cut -c100-160)" | tee -a gpurun_out/s_gatys_sweep.txt
done
