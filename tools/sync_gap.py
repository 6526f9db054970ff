#!/usr/bin/env python3
"""Idle gaps (> 15 us) between consecutive kernels of the last bench step in a rocprofv3 kernel trace: where the GPU
waits for the host (synthesize's host sync). Usage: python tools/sync_gap.py TRACE_DIR [launches per step]"""
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 711
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))[-n:]
prev = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if prev and s - prev[1] > 15000:
        print(f"{(s - prev[1]) / 1e3:8.1f} us  after {prev[0][:50]}  before {r['Kernel_Name'][:50]}")
    prev = (r["Kernel_Name"], e)
print(f"span {(int(rows[-1]['End_Timestamp']) - int(rows[0]['Start_Timestamp'])) / 1e6:.3f} ms")
