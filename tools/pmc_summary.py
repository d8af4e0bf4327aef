"""Per-kernel summary of tools/prof_pass.sh output (rocprofv3 CSV), averaged over dispatches.

  python tools/pmc_summary.py gpurun_out/<tag> [--json out.json] [--res-json profiles/pmc_res_conv.json]

Prints per kernel: average duration (kernel-trace pass), every PMC counter averaged over its
dispatches, and derived figures: HBM bytes (gfx950 correction: 2*FETCH_SIZE + WRITE_SIZE, KiB;
MI355X_MICROARCH.md HBM section), MFMA busy fraction, effective clock from GRBM_GUI_ACTIVE/8.
Scratch analysis tool, not part of the product."""
import collections
import csv
import glob
import json
import os
import re
import sys


_TARG = {"DF16b": "bf16", "DF16_": "fp16", "f": "float"}


def pretty(k):
    """hipcc leaves the _Float16/__bf16 template kernels mangled in the trace: _ZN3nst12wstat_kernelIDF16bLi8ELi0ELb0ELb0EE...
    -> 'nst::wstat_kernel<bf16, 8, 0, false, false>'"""
    m = re.match(r"_ZN3nst(\d+)(\w+?)I((?:DF16b|DF16_|f|Li-?\d+E|Lb[01]E)+)EEvNS_10ConvParamsE", k)
    if not m or len(m.group(2)) != int(m.group(1)):
        return k
    args = []
    for a in re.findall(r"DF16b|DF16_|f(?!\w)|Li-?\d+E|Lb[01]E|f", m.group(3)):
        if a in _TARG:
            args.append(_TARG[a])
        elif a.startswith("Li"):
            args.append(a[2:-1])
        else:
            args.append("true" if a[2] == "1" else "false")
    return f"nst::{m.group(2)}<{', '.join(args)}>"


def short(k):
    k = pretty(k)
    m = re.search(r"conv_kernelI(DF16b|f)Li(\d)ELi(\d)ELi(\d)ELi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELi(\d)ELi(\d)ELi(\d)ELi(\d)ELi(\d)E", k)
    if m:
        t, mode, ks, s, ci, bn, th, tw, wm, wn, ink, outk, var = m.groups()
        return f"conv{'b' if t == 'DF16b' else 'f'} md{mode} k{ks}s{s} ci{ci} bn{bn} {th}x{tw} w{wm}x{wn} in{ink} out{outk} v{var}"
    m = re.search(r"conv_kernel<[^>]*>", k)
    if m:
        return m.group(0)[:90]
    return re.sub(r"\(.*", "", k)[:70]


def load(d):
    dur = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "stats", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[pretty(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    ctr = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    for f in glob.glob(os.path.join(d, "*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ctr[pretty(r["Kernel_Name"])][r["Counter_Name"]][(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
    return dur, ctr


def main():
    d = sys.argv[1]
    dur, ctr = load(d)
    out = {}
    names = sorted(set(dur) | set(ctr), key=lambda k: -sum(dur.get(k, [0])))
    for k in names:
        if "copyBuffer" in k or "fillBuffer" in k:
            continue
        ds = dur.get(k, [])
        rec = {"launches_traced": len(ds), "avg_us": (sum(ds) / len(ds) / 1e3) if ds else None,
               "total_us": sum(ds) / 1e3}
        for c, per in ctr.get(k, {}).items():
            rec[c] = sum(per.values()) / len(per)
        if "FETCH_SIZE" in rec and "WRITE_SIZE" in rec:
            rec["hbm_bytes"] = (2 * rec["FETCH_SIZE"] + rec["WRITE_SIZE"]) * 1024
        if "GRBM_GUI_ACTIVE" in rec and rec.get("avg_us"):
            rec["eff_clock_ghz"] = rec["GRBM_GUI_ACTIVE"] / 8 / (rec["avg_us"] * 1e3)
        out[k] = rec
        print(f"== {short(k)}   avg {rec['avg_us'] or 0:.1f} us x{len(ds)}")
        print("   " + "  ".join(f"{c.replace('SQ_', '')}={v:.4g}" for c, v in sorted(rec.items())
                              if c not in ("launches_traced", "avg_us", "total_us") and v is not None))
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
            json.dump(out, f, indent=1)
    if "--res-json" in sys.argv:  # the dominant kernel's summary bench.py reads (keyed by the library build)
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from neuralstyletransferv1_amd._lib import trunk_kernel_sha
        key = next(k for k in out if "wst16_kernel<bf16, 8, 0, false, false>" in k)
        r = out[key]
        res = {
            "source": f"tools/prof_pass.sh {os.path.basename(d.rstrip('/'))} (rocprofv3 --kernel-trace --stats, then "
                      "--pmc passes in separate runs of bench.py)",
            "units": "hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950: FETCH_SIZE counts half of a wide "
                     "coalesced read stream, MI355X_MICROARCH.md HBM section)",
            "kernel_src_sha16": trunk_kernel_sha(),
            "res_conv_kernel": key,
            "hbm_bytes_per_launch": r.get("hbm_bytes"),
            "fetch_size_kib": r.get("FETCH_SIZE"),
            "write_size_kib": r.get("WRITE_SIZE"),
            "avg_us_profiled": r.get("avg_us"),
            "eff_clock_ghz": r.get("eff_clock_ghz"),
            "mfma_insts_per_launch": r.get("SQ_INSTS_MFMA"),
            "algorithmic_bytes_per_launch": 530841600,
        }
        jk = next((k for k in out if "wst16_kernel<bf16, 8, 2, false, false>" in k), None)
        if jk is not None:  # the joined variant (residual join in the fill), same PMC passes
            j = out[jk]
            res["joined"] = {"kernel": jk, "avg_us_profiled": j.get("avg_us"), "hbm_bytes_per_launch": j.get("hbm_bytes"),
                             "eff_clock_ghz": j.get("eff_clock_ghz"), "algorithmic_bytes_per_launch": 2 * 530841600}
        # NST_DT_F16M's dominant kernel (the split-operand conv2, fp32 operand and output), same passes
        from neuralstyletransferv1_amd._lib import ws2_kernel_sha
        mk = next((k for k in out if re.search(r"ws2_kernel<fp16, 32, 64, \d+, false, \d, true, true", k)), None)
        if mk is not None:
            m = out[mk]
            res["fp16m_conv2"] = {"kernel": mk, "kernel_src_sha16": ws2_kernel_sha(), "avg_us_profiled": m.get("avg_us"),
                                  "hbm_bytes_per_launch": m.get("hbm_bytes"), "eff_clock_ghz": m.get("eff_clock_ghz")}
        with open(sys.argv[sys.argv.index("--res-json") + 1], "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
