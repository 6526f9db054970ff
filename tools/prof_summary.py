"""Summarise a rocprofv3 kernel-trace CSV of bench.py: one synthesis step split into its components
(text encoder | index path | CFM decoder | vocoder | denoiser) by boundary kernels, then the top kernels.
Usage: python tools/prof_summary.py kernel_trace.csv [TOP]"""
import csv
import subprocess
import sys
from collections import defaultdict

path = sys.argv[1]
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r['Start_Timestamp']))


def dur(r):
    return (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6


def short(n):
    try:
        d = subprocess.run(['c++filt', n], capture_output=True, text=True).stdout.strip()
    except Exception:
        d = n
    d = d.replace('mt::', '').replace('ConvArgs', '').replace('__hip_bfloat16', 'bf16')
    return d[:110]


starts = [i for i, r in enumerate(rows) if 'embed_kernel' in r['Kernel_Name']]
s, e = starts[-2], starts[-1]  # the last full step before the final one
step = rows[s:e]
span = (int(step[-1]['End_Timestamp']) - int(step[0]['Start_Timestamp'])) / 1e6
busy = sum(dur(r) for r in step)
print(f"step span {span:.2f} ms, kernel busy {busy:.2f} ms, launches {len(step)}")
# components by boundary kernels (in launch order)
comp, cur = defaultdict(lambda: [0.0, 0, None, None]), 'encoder'
for r in step:
    k = r['Kernel_Name']
    if 'durations_kernel' in k:
        cur = 'index path'
    elif cur == 'index path' and ('sinus_kernel' in k):
        cur = 'decoder'
    elif 'denorm_crop_kernel' in k:
        cur = 'denorm'
    elif cur == 'denorm' and 'bct_to_btc' in k:
        cur = 'vocoder'
    elif 'stft_denoise' in k:
        cur = 'denoiser'
    c = comp[cur]
    c[0] += dur(r)
    c[1] += 1
    t0, t1 = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    c[2] = t0 if c[2] is None else min(c[2], t0)
    c[3] = t1 if c[3] is None else max(c[3], t1)
for name, (ms, n, t0, t1) in comp.items():
    print(f"  {name:11s} busy {ms:7.2f} ms  span {(t1 - t0) / 1e6:7.2f} ms  {n:4d} launches")
byname = defaultdict(lambda: [0.0, 0])
for r in step:
    byname[r['Kernel_Name']][0] += dur(r)
    byname[r['Kernel_Name']][1] += 1
for k, v in sorted(byname.items(), key=lambda x: -x[1][0])[:int(sys.argv[2]) if len(sys.argv) > 2 else 30]:
    print(f"{v[0]:8.2f} ms {v[1]:5d} x  {short(k)}")
