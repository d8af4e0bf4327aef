set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
export NST_HIP_LIB=$PWD/sweep/libnst_hip_th6.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_layers.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/w4.log 2>&1
tail -45 gpurun_out/w4.log | cut -c1-300
