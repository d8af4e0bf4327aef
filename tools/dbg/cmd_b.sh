set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 200 python -u tools/dbg/f16m_conv1.py > gpurun_out/dbg_f16m.txt 2>&1; cat gpurun_out/dbg_f16m.txt | grep -v amdgpu.ids
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -k "not fp16m" > gpurun_out/gpu_tests_r04b.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/gpu_tests_r04b.log | head -20; tail -5 gpurun_out/gpu_tests_r04b.log; exit 1; }
tail -2 gpurun_out/gpu_tests_r04b.log
