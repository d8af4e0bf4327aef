set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/r1_gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/r1_gpu_tests.log | head -20; tail -2 gpurun_out/r1_gpu_tests.log
case $rc in 124|137|134|139) exit 1;; esac
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1_smoke.log 2>&1; echo "smoke rc=$?"; tail -3 gpurun_out/r1_smoke.log
