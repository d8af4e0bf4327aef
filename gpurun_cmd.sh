# GPU validation: parity tests, then the bench (each step under its own time limit, stop at first failure)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${TESTSEL:-} > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 ${BENCHARGS:-} > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('fps', d['value'], 'ms', d['ms_per_step'], 'res', d['roofline']['avg_launch_ms'], d['whole_path']['per_layer_avg_ms'], 'ssim', d.get('ssim_vs_cpu'))"
