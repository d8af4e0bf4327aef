set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layers.py -m gpu -q --timeout 300 --timeout-method thread -k "range_check or reconet" > gpurun_out/v_tests.log 2>&1; echo "tests rc=$?"; grep -E "FAILED|passed|failed" gpurun_out/v_tests.log | head -5
timeout -k 10 120 python -u tools/mode_profile.py bf16 reconet > gpurun_out/v_r.log 2>&1; tail -1 gpurun_out/v_r.log | cut -c1-200
