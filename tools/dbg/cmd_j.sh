set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
: > gpurun_out/j_sweep.txt
for F in 0x1ffc 0x1ff0 0x1f00; do
  for B in 0x1ffc 0x1ff0 0x1f00 0x1000; do
    NST_VGG_GEMM_F=$F NST_VGG_GEMM_B=$B GATYS_STEPS=100 timeout -k 10 120 python -u tools/gatys_bench.py > gpurun_out/j_one.log 2>&1
    rc=$?
    echo "F=$F B=$B rc=$rc $(tail -1 gpurun_out/j_one.log | cut -c1-200)" | tee -a gpurun_out/j_sweep.txt
    case $rc in 0) ;; *) exit 1;; esac
  done
done
