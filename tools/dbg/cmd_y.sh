set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layers.py tests/test_gpu_pipeline.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/y_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "FAILED|passed|failed|Error" gpurun_out/y_tests.log | head -8
case $rc in 124|137|134|139) exit 1;; esac
for a in reconet reconet_frn; do timeout -k 10 120 python -u tools/mode_profile.py bf16 $a > gpurun_out/y_p_$a.log 2>&1 || exit 1; tail -1 gpurun_out/y_p_$a.log | cut -c1-150; done
timeout -k 10 120 python -u tools/mode_profile.py fp32 johnson > gpurun_out/y_p_j32.log 2>&1 || exit 1; tail -1 gpurun_out/y_p_j32.log | cut -c1-150
