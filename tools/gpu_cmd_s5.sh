set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u tools/dbg_ws.py > gpurun_out/dbg_ws5.txt 2>&1; echo "ws rc=$?"; grep -c deterministic gpurun_out/dbg_ws5.txt; grep DEPENDS gpurun_out/dbg_ws5.txt | head
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_s5.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_s5.log | head -20; tail -20 gpurun_out/gpu_tests_s5.log; exit 1; }
tail -1 gpurun_out/gpu_tests_s5.log
bash tools/gpu_aux.sh r03_s5
