set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/abn.sh 2 default th6 th8 2>&1 | sed 's/| per-8-frames ms: .*deconv1=\([0-9.]*\) deconv2=\([0-9.]*\).*/deconv1=\1 deconv2=\2/'
for L in th6 th8; do
  export NST_HIP_LIB=$PWD/sweep/libnst_hip_$L.so
  echo "== tests $L"
  timeout -k 10 300 python -u -m pytest tests/test_gpu_layers.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -2
done
