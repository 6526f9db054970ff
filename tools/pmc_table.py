#!/usr/bin/env python3
"""Per-kernel table from tools/pmc.sh passes: launch time, clock, MFMA-busy fraction, VALU / LDS instructions
per wave, HBM bytes per launch.
Clock: GRBM_GUI_ACTIVE / 8 XCDs / kernel time is the in-kernel clock only for dispatches of >= 0.3 ms
(MI355X_MICROARCH.md, 'DVFS give-back': the quotient reads high on shorter ones, up to 3x here); shorter kernels get
the median clock of the run's long dispatches (column src 'run'), and every clock is capped at the 2.4 GHz maximum.
MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES (summed over the 1,024 SIMDs) / (kernel time x that clock x 1024).
Usage: python tools/pmc_table.py gpurun_out/TAG > table.txt"""
import csv
import glob
import os
import subprocess
import sys
from collections import defaultdict

root = sys.argv[1]
agg = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = (r["Kernel_Name"], int(r["Grid_Size"]))
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if r["Counter_Name"] in ("SQ_WAVES", "FETCH_SIZE"):
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)


def short(n):
    try:
        n = subprocess.run(["c++filt", n], capture_output=True, text=True).stdout.strip()
    except Exception:
        pass
    return n.replace("mt::", "").replace("(VConvArgs)", "").replace("(VPairArgs)", "").replace("void ", "")[:48]


print(f"{'kernel':48s} {'grid':>7s} {'n':>4s} {'us':>7s} {'GHz':>5s} {'src':>4s} {'mfma':>5s} {'valu/w':>8s} "
      f"{'lds/w':>7s} {'fetchMB':>8s} {'writeMB':>8s}")
LONG_US, FMAX = 300.0, 2.4


def mean(v):
    return sum(v) / len(v) if v else 0.0


long_clk = []
for k, cs in agg.items():
    us = mean(dur[k])
    g = mean(cs.get("GRBM_GUI_ACTIVE", []))
    if us >= LONG_US and g:
        long_clk.append(g / 8 / (us * 1e3))
f_run = sorted(long_clk)[len(long_clk) // 2] if long_clk else 2.1
for k, cs in sorted(agg.items(), key=lambda kv: -sum(dur[kv[0]])):
    m = {c: mean(v) for c, v in cs.items()}
    us = mean(dur[k])
    g = m.get("GRBM_GUI_ACTIVE", 0)
    own = g / 8 / (us * 1e3) if us and g else 0.0
    ghz, src = (min(own, FMAX), "own") if us >= LONG_US else (min(f_run, FMAX), "run")
    mf = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (us * 1e3 * ghz * 1024) if us and ghz else 0
    w = m.get("SQ_WAVES", 1)
    print(f"{short(k[0]):48s} {k[1]:7d} {len(dur[k]):4d} {us:7.1f} {ghz:5.2f} {src:>4s} {mf:5.2f} "
          f"{m.get('SQ_INSTS_VALU', 0) / w:8.0f} {m.get('SQ_INSTS_LDS', 0) / w:7.0f} "
          f"{2 * m.get('FETCH_SIZE', 0) / 1024:8.1f} {m.get('WRITE_SIZE', 0) / 1024:8.1f}")
