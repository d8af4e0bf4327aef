set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 120 python -u tools/mode_profile.py bf16 reconet 2>/dev/null | tail -1
timeout -k 10 120 python -u tools/mode_profile.py bf16 johnson 2>/dev/null | tail -1
