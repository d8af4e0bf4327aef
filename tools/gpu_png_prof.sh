set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/png_prof_b -o run -- python3 tools/png_bench.py --reps 5 > gpurun_out/png_prof_b.log 2>&1 || { tail -20 gpurun_out/png_prof_b.log; exit 1; }
f=$(find gpurun_out/png_prof_b -name "*kernel_stats.csv" | head -1); grep -E "png_" "$f" | cut -c1-200
