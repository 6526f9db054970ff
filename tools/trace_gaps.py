#!/usr/bin/env python3
"""Idle time inside one bench step of a rocprofv3 kernel trace: the gaps between consecutive kernels (end of one to
start of the next), summed, and the largest ones with the kernels on either side.
Usage: python tools/trace_gaps.py kernel_trace.csv [TOP]"""
import csv
import subprocess
import sys

path = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 15
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "embed_kernel" in r["Kernel_Name"]]
s, e = starts[-2], starts[-1]
step = rows[s:e]


def short(n):
    try:
        d = subprocess.run(["c++filt", n], capture_output=True, text=True).stdout.strip()
    except Exception:
        d = n
    return d.replace("mt::", "").replace("__hip_bfloat16", "bf16")[:60]


gaps = []
for a, b in zip(step, step[1:]):
    g = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3
    gaps.append((g, short(a["Kernel_Name"]), short(b["Kernel_Name"])))
pos = [g for g in gaps if g[0] > 0]
print(f"{len(step)} launches, idle {sum(g[0] for g in pos) / 1e3:.3f} ms in {len(pos)} gaps "
      f"(> 5 us: {sum(g[0] for g in pos if g[0] > 5) / 1e3:.3f} ms in {sum(1 for g in pos if g[0] > 5)})")
for g, a, b in sorted(pos, reverse=True)[:top]:
    print(f"  {g:8.1f} us  {a}  ->  {b}")
