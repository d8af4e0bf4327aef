set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/abn.sh 1 default r3 r1 nw8 th16 default 2>&1 | sed 's/| per-8-frames ms: conv1=\([0-9.]*\) .*/conv1=\1/'
for L in r3 nw8 th16; do
  export NST_HIP_LIB=$PWD/sweep/libnst_hip_$L.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_layers.py -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -1
done
