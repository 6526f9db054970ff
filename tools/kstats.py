#!/usr/bin/env python3
"""Average launch time per kernel from a rocprofv3 --stats output directory (its *kernel_stats.csv), sorted by total
time. Usage: python tools/kstats.py DIR [REGEX]"""
import csv
import glob
import os
import re
import sys

d = sys.argv[1]
rx = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
fs = [d] if d.endswith(".csv") else glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
if not fs:
    sys.exit(f"no kernel_stats.csv under {d}")
rows = list(csv.DictReader(open(fs[0])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows:
    n = r["Name"].replace("void ", "").replace("mt::", "").replace("(mt::VPairArgs)", "").replace("(mt::VConvArgs)", "")
    if rx and not rx.search(n):
        continue
    print(f"{float(r['TotalDurationNs']) / 1e6:9.3f} ms {int(r['Calls']):5d} x {float(r['AverageNs']) / 1e3:9.1f} us  {n[:70]}")
