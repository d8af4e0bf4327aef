"""Per-kernel PMC summary of rocprofv3 runs (sqlite rocpd output or CSV), averaged over dispatches.
Scratch tool: python tools_pmc_summary.py gpurun_out/pmc1 gpurun_out/pmc2 ..."""
import collections, csv, glob, os, re, sqlite3, sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for d in sys.argv[1:]:
    dbs = glob.glob(os.path.join(d, "*.db"))
    if dbs:
        c = sqlite3.connect(dbs[0])
        per = collections.defaultdict(float)
        for disp, name, cn, v, st, en in c.execute(
                "select dispatch_id, kernel_name, counter_name, value, start, end from counters_collection"):
            per[(disp, name, cn)] += v
            dur[(name, d)].append((disp, en - st))
        for (disp, name, cn), v in per.items():
            agg[name][cn].append(v)
    else:
        for r in csv.DictReader(open(f"{d}/b_counter_collection.csv")):
            agg[r['Kernel_Name']][r['Counter_Name']].append(float(r['Counter_Value']))


def short(k):
    m = re.search(r'conv_kernelI(DF16b|f)Li(\d)ELi(\d)ELi(\d)ELi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)', k)
    if m:
        return f"conv{'b' if m.group(1) == 'DF16b' else 'f'} m{m.group(2)} k{m.group(3)} s{m.group(4)} ci{m.group(5)} bn{m.group(6)} th{m.group(7)} tw{m.group(8)}"
    return k[:48]


for k, cs in agg.items():
    if 'copyBuffer' in k:
        continue
    ds = {}
    for (name, d), lst in dur.items():
        if name == k:
            for disp, t in lst:
                ds[(d, disp)] = t
    avg = sum(ds.values()) / max(len(ds), 1) / 1e3
    v = {c: sum(x) / len(x) for c, x in cs.items()}
    print(f"== {short(k)}  avg {avg:.1f} us  dispatches {len(ds)}")
    print("   " + "  ".join(f"{c.replace('SQ_', '')}={v[c]:.3g}" for c in sorted(v)))
