#!/bin/bash
# Beyond-configs[1] measurements in one call: Gatys 512^2 Adam step (+ rocprofv3 stats of it), per-architecture
# frames/s, configs[4] mask step, the CLI with host PNG/JPEG I/O, the post chain.  Each step under its own limit.
#   bash tools/gpu_aux.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-aux}
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || { echo "bench failed"; tail -30 gpurun_out/bench_$T.err; exit 1; }
python tools/bench_brief.py gpurun_out/bench_$T.json
timeout -k 10 200 python -u tools/batch_sweep.py 8 4 2 1 > gpurun_out/batch_$T.txt 2>&1 || { tail -20 gpurun_out/batch_$T.txt; exit 1; }
grep batch gpurun_out/batch_$T.txt
GATYS_STEPS=100 timeout -k 10 240 python -u tools/gatys_bench.py > gpurun_out/gatys_$T.json 2> gpurun_out/gatys_$T.err || { tail -20 gpurun_out/gatys_$T.err; exit 1; }
cat gpurun_out/gatys_$T.json
GATYS_STEPS=30 timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gatys_$T -o gatys -- python3 tools/gatys_bench.py > gpurun_out/prof_gatys_$T.log 2>&1 || { echo "gatys prof failed"; tail -20 gpurun_out/prof_gatys_$T.log; exit 1; }
timeout -k 10 300 python -u tools/arch_bench.py > gpurun_out/arch_$T.txt 2>&1 || { tail -20 gpurun_out/arch_$T.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/arch_$T.txt
timeout -k 10 300 python -u tools/seg_bench.py > gpurun_out/seg_$T.json 2> gpurun_out/seg_$T.err || { tail -20 gpurun_out/seg_$T.err; exit 1; }
tail -3 gpurun_out/seg_$T.json
timeout -k 10 400 python -u tools/cli_bench.py --frames 48 > gpurun_out/cli_$T.json 2> gpurun_out/cli_$T.err || { tail -20 gpurun_out/cli_$T.err; exit 1; }
tail -3 gpurun_out/cli_$T.json
timeout -k 10 200 python -u tools/post_bench.py > gpurun_out/post_$T.txt 2>&1 || { echo "post bench failed"; tail -5 gpurun_out/post_$T.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/post_$T.txt | tail -30
