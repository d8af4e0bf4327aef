set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/abn.sh 3 default pack 2>&1
export NST_HIP_LIB=$PWD/sweep/libnst_hip_pack.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_layers.py -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -2
