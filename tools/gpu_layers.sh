set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_layers.py -x -v -s --timeout 400 --timeout-method thread > gpurun_out/layers.log 2>&1; echo "layers rc=$?"
tail -5 gpurun_out/layers.log
