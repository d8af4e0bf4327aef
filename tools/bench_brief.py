"""One-line summary of a bench.py JSON line (scratch helper for GPU runs)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
wp = d["whole_path"]
print("fps", d["value"], "ms/step", d["ms_per_step"], "trunk", d["roofline"]["avg_launch_ms"], "frac", d["roofline"]["frac"],
      "joined", wp["trunk_joined_avg_ms"], "conv/step", wp["conv_kernel_ms_per_step"])
print(" ".join(f"{k.split('.')[0]}{'.' + k.split('.')[1] if k.startswith('res') else ''}={v:.3f}"
               for k, v in wp["per_layer_avg_ms"].items()))
for k in ("fp32_parity_frames_per_s", "ssim_vs_cpu", "max_abs_lsb_vs_cpu", "within_2lsb_vs_cpu"):
    if k in d:
        print(k, d[k])
if d.get("cpu_baseline"):
    print("cpu", json.dumps(d["cpu_baseline"]))
for k in ("fp16_mode", "fp16m_mode", "fp32s_mode", "gpu_full_chain", "gpu_png_encode"):
    if d.get(k):
        print(k, json.dumps(d[k]))
if "measured_peak" in d["roofline"]:
    print("frac_of_measured", d["roofline"].get("frac_of_measured_peak"), "joined", json.dumps(d["roofline"].get("joined")))
