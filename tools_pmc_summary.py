import csv, collections, sys, glob
agg = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for d in sys.argv[1:]:
    for r in csv.DictReader(open(f"{d}/b_counter_collection.csv")):
        agg[r['Kernel_Name']][r['Counter_Name']].append(float(r['Counter_Value']))
    for r in csv.DictReader(open(f"{d}/b_kernel_trace.csv")):
        dur[r['Kernel_Name']].append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
def short(k):
    import re
    m = re.search(r'conv_kernelI(DF16b|f)Li(\d)ELi(\d)ELi(\d)ELi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)', k)
    if m: return f"conv{'b' if m.group(1)=='DF16b' else 'f'} m{m.group(2)} k{m.group(3)} s{m.group(4)} ci{m.group(5)} bn{m.group(6)} th{m.group(7)} tw{m.group(8)}"
    return k[:40]
for k, cs in agg.items():
    if 'copyBuffer' in k: continue
    d = sum(dur[k]) / len(dur[k]) / 1e3
    v = {c: sum(x) / len(x) for c, x in cs.items()}
    print(f"== {short(k)}  avg {d:.1f} us  calls {len(dur[k])}")
    print("   " + "  ".join(f"{c.replace('SQ_','')}={v[c]:.3g}" for c in sorted(v)))
