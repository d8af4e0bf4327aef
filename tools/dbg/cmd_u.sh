set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
: > gpurun_out/u_ksel.txt
for k in "" no_wstat no_ws2 no_wphase no_ws9 no_kyrot; do
  MODE_KSEL=$k timeout -k 10 120 python -u tools/mode_profile.py bf16 johnson > gpurun_out/u_one.log 2>&1 || exit 1
  tail -1 gpurun_out/u_one.log | tee -a gpurun_out/u_ksel.txt | cut -c1-200
done
for v in tr42 c1w c1x; do NST_HIP_LIB=sweep/libnst_hip_$v.so timeout -k 10 120 python -u tools/mode_profile.py bf16 reconet > gpurun_out/u_r.log 2>&1 || exit 1; tail -1 gpurun_out/u_r.log | tee -a gpurun_out/u_ksel.txt | cut -c1-300; done
timeout -k 10 120 python -u tools/mode_profile.py bf16 reconet > gpurun_out/u_r.log 2>&1 || exit 1; tail -1 gpurun_out/u_r.log | tee -a gpurun_out/u_ksel.txt | cut -c1-300
