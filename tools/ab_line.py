"""One summary line of a tools/mode_profile.py JSON for A/B scripts: variant, frames/s, per-layer ms (short names)."""
import json
import sys

d = json.load(open(sys.argv[2]))
L = d["per_layer_ms"]
short = {k: k.replace("encoder.layers.", "e").replace("decoder.layers.", "d").replace(".layers.0.layers.1", "")
         .replace(".branch.", "b") for k in L}
print(sys.argv[1], d["frames_per_s"], " ".join(f"{short[k]}={v:.3f}" for k, v in L.items()))
