#!/bin/bash
# Bench each variant library (build/variants/*/libnst_hip.so) plus the default one; per-layer times.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/sweep
for lib in neuralstyletransferv1_amd/libnst_hip.so build/variants/*/libnst_hip.so; do
  [ -f "$lib" ] || continue
  name=$(basename $(dirname $lib))
  NST_HIP_LIB=$PWD/$lib timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/sweep/$name.json 2> gpurun_out/sweep/$name.err || { echo "$name failed"; tail -5 gpurun_out/sweep/$name.err; exit 1; }
  python -c "
import json
d = json.loads(open('gpurun_out/sweep/$name.json').read().strip().splitlines()[-1])
l = d['whole_path']['per_layer_avg_ms']
print('$name', d['value'], ' '.join(f'{k.split(\".\")[0]}={v:.3f}' for k, v in l.items() if not k.startswith('res')),
      'trunk', d['roofline']['avg_launch_ms'], 'joined', d['whole_path'].get('trunk_joined_avg_ms'))"
done
