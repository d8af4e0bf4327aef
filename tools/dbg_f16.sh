cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u tools/dbg_f16.py reconet_frn tests/golden/model_reconet_frn_s1_48x84.npz > gpurun_out/dbg_frn.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/dbg_f16.py reconet tests/golden/model_reconet_s1_48x84.npz > gpurun_out/dbg_rec.txt 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s -k "fp32s" --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r03s.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_r03s.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_deeplab.py tests/test_gpu_flow.py -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r03b.log 2>&1
tail -3 gpurun_out/gpu_tests_r03b.log
