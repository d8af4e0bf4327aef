set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gatys.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/t_tests.log 2>&1; echo "gatys tests rc=$?"; tail -2 gpurun_out/t_tests.log
: > gpurun_out/t_gatys_sweep.txt
for m in "X=0" "NST_VGG_GEMM_F=0x0 NST_VGG_GEMM_B=0x0" "NST_VGG_GEMM_F=0x1000 NST_VGG_GEMM_B=0x0" "X=0"; do
  env $m GATYS_STEPS=300 timeout -k 10 120 python -u tools/gatys_bench.py > gpurun_out/t_one.log 2>&1 || exit 1
  echo "$m $(tail -1 gpurun_out/t_one.log | cut -c100-160)" | tee -a gpurun_out/t_gatys_sweep.txt
done
tail -1 gpurun_out/t_one.log > gpurun_out/t_gatys.json
SEG_GRAPH=1 SEG_DTYPES=fp32s timeout -k 10 300 python -u tools/seg_bench.py > gpurun_out/t_seg.log 2>&1; echo "seg rc=$?"; tail -1 gpurun_out/t_seg.log | cut -c1-900
