set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_pipeline_golden.py -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r06_e.log 2>&1; rc=$?
grep -E "vs reference file|passed|failed|Error" gpurun_out/gpu_tests_r06_e.log | tail -60
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
for i in 1 2; do
 echo "== default"; timeout -k 10 120 python -u tools/batch_sweep.py 8 2>&1 | grep -v amdgpu.ids || exit 1
 echo "== coal"; NST_HIP_LIB=$PWD/neuralstyletransferv1_amd/libnst_hip_coal.so timeout -k 10 120 python -u tools/batch_sweep.py 8 2>&1 | grep -v amdgpu.ids || exit 1
done
