#!/bin/bash
# Samples the GPU's power and clocks (amd-smi metric, read-only) idle and while tools/power_load.py runs the
# configs[1] bf16 batch back to back, to test whether the step is power-limited.
#   bash tools/power_probe.sh
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
timeout -k 10 60 amd-smi metric -p -c > gpurun_out/power_idle.txt 2>&1
timeout -k 10 150 python -u tools/power_load.py 50 > gpurun_out/power_load.txt 2>&1 &
pid=$!
sleep 35
for i in 1 2 3 4 5; do
  timeout -k 5 20 amd-smi metric -p -c > gpurun_out/power_busy_$i.txt 2>&1
  sleep 1
done
wait $pid
rc=$?
cat gpurun_out/power_load.txt
echo "load rc=$rc"
exit $rc
