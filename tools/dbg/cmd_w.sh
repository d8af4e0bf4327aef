set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layers.py -m gpu -q -x --timeout 300 --timeout-method thread -k "reconet or ws9 or fp16m or small or 1080p" > gpurun_out/w_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "FAILED|passed|failed|Error" gpurun_out/w_tests.log | head -8
case $rc in 124|137|134|139) exit 1;; esac
for a in reconet reconet_frn; do for d in bf16 fp16; do timeout -k 10 120 python -u tools/mode_profile.py $d $a > gpurun_out/w_$a_$d.log 2>&1 || exit 1; tail -1 gpurun_out/w_$a_$d.log | cut -c1-170; done; done
timeout -k 10 120 python -u tools/mode_profile.py bf16 johnson > gpurun_out/w_j.log 2>&1 || exit 1; tail -1 gpurun_out/w_j.log | cut -c1-200
