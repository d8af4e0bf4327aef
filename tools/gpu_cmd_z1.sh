set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -3
timeout -k 10 400 python -u bench.py > gpurun_out/bench_z1.json 2> gpurun_out/bench_z1.err || { echo "bench failed"; tail -20 gpurun_out/bench_z1.err; exit 1; }
python tools/bench_brief.py gpurun_out/bench_z1.json | head -3
