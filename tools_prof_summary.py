"""Summarise a rocprofv3 kernel-trace CSV: per-synthesize-step time by kernel class and top kernels."""
import csv, re, subprocess, sys
from collections import defaultdict
path = sys.argv[1]
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r['Start_Timestamp']))
def dur(r): return (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6
def short(n):
    try: d = subprocess.run(['c++filt', n], capture_output=True, text=True).stdout.strip()
    except Exception: d = n
    d = d.replace('mt::', '').replace('ConvArgs', '').replace('__hip_bfloat16', 'bf16')
    return d[:110]
starts = [i for i, r in enumerate(rows) if 'durations_kernel' in r['Kernel_Name']]
s, e = starts[-2], starts[-1]   # last full step before the final (roofline) one
agg = defaultdict(lambda: [0.0, 0])
for r in rows[s:e]:
    k = r['Kernel_Name']; g = (r['Grid_Size_X'], r['Grid_Size_Y'], r['Workgroup_Size_X'])
    agg[(k, g)][0] += dur(r); agg[(k, g)][1] += 1
span = (int(rows[e-1]['End_Timestamp']) - int(rows[s]['Start_Timestamp'])) / 1e6
busy = sum(v[0] for v in agg.values())
print(f"step span {span:.2f} ms, kernel busy {busy:.2f} ms, launches {e-s}")
byname = defaultdict(lambda: [0.0, 0])
for (k, g), v in agg.items(): byname[k][0] += v[0]; byname[k][1] += v[1]
for k, v in sorted(byname.items(), key=lambda x: -x[1][0])[:int(sys.argv[2]) if len(sys.argv) > 2 else 20]:
    print(f"{v[0]:8.2f} ms {v[1]:5d} x  {short(k)}")
