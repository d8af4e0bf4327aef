set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m cProfile -o gpurun_out/cli.prof tools/cli_bench.py --frames 48 > gpurun_out/cli_c1.txt 2>&1 || { tail -20 gpurun_out/cli_c1.txt; exit 1; }
tail -3 gpurun_out/cli_c1.txt
python -c "
import pstats; p=pstats.Stats('gpurun_out/cli.prof'); p.sort_stats('cumulative').print_stats(45)" 2>&1 | tail -60
