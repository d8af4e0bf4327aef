#!/bin/bash
# Socket power and clocks (amd-smi metric, read-only) for each precision mode / network under a 30 s back-to-back run
# of the configs[1] batch; one line per configuration: frames/s, mean W, mean GFX MHz, J per frame.
#   bash tools/power_modes.sh
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
for cfg in "johnson bf16" "johnson fp16" "johnson fp16m" "johnson fp32s" "reconet bf16"; do
  set -- $cfg
  tag=$1_$2
  timeout -k 10 120 python -u tools/power_load.py 30 $1 $2 > gpurun_out/pm_load_$tag.txt 2>&1 &
  pid=$!
  sleep 24
  for i in 1 2 3; do timeout -k 5 20 amd-smi metric -p -c > gpurun_out/pm_${tag}_$i.txt 2>&1; sleep 1; done
  wait $pid || { echo "$tag load failed"; cat gpurun_out/pm_load_$tag.txt | tail -5; exit 1; }
  python3 - "$tag" <<'PY'
import re, sys, glob
tag = sys.argv[1]
load = open(f"gpurun_out/pm_load_{tag}.txt").read()
fps = float(re.search(r"([\d.]+) frames/s", load.split("load done:")[1]).group(1))
w, mhz = [], []
for f in sorted(glob.glob(f"gpurun_out/pm_{tag}_[0-9].txt")):
    t = open(f).read()
    w.append(float(re.search(r"SOCKET_POWER: (\d+)", t).group(1)))
    mhz += [float(v) for v in re.findall(r"GFX_\d+:\s+CLK: (\d+) MHz", t)]
W = sum(w) / len(w)
print(f"{tag}: {fps:.1f} frames/s, {W:.0f} W, GFX {sum(mhz) / len(mhz):.0f} MHz, {W / fps:.3f} J/frame")
PY
done
