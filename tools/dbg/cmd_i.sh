set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
SEG_STEPS=3 SEG_DTYPES=fp32s SEG_MASK_DT=fp32s timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/i_seg -o run -- python3 tools/seg_bench.py > gpurun_out/i_seg.log 2>&1 || { echo "seg prof failed"; tail gpurun_out/i_seg.log; exit 1; }
echo seg ok
GATYS_STEPS=20 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/i_gatys -o run -- python3 tools/gatys_bench.py > gpurun_out/i_gatys.log 2>&1 || { echo "gatys prof failed"; tail gpurun_out/i_gatys.log; exit 1; }
echo gatys ok
bash tools/prof_pass.sh prof_r04_i1
