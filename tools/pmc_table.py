#!/usr/bin/env python3
"""Per-kernel table from tools/pmc.sh passes: launch time, XCD clock, MFMA-busy fraction, VALU / LDS instructions
per wave, HBM bytes per launch. MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)
(GRBM_GUI_ACTIVE sums the 8 XCDs' GPU-busy cycles; MFMA-busy cycles sum over every SIMD).
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


print(f"{'kernel':48s} {'grid':>7s} {'n':>4s} {'us':>7s} {'GHz':>5s} {'mfma':>5s} {'valu/w':>8s} {'lds/w':>7s} "
      f"{'fetchMB':>8s} {'writeMB':>8s}")
for k, cs in sorted(agg.items(), key=lambda kv: -sum(dur[kv[0]])):
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    us = sum(dur[k]) / max(1, len(dur[k]))
    g = m.get("GRBM_GUI_ACTIVE", 0)
    ghz = g / 8 / (us * 1e3) if us else 0
    mf = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (g / 8 * 1024) if g else 0
    w = m.get("SQ_WAVES", 1)
    print(f"{short(k[0]):48s} {k[1]:7d} {len(dur[k]):4d} {us:7.1f} {ghz:5.2f} {mf:5.2f} "
          f"{m.get('SQ_INSTS_VALU', 0) / w:8.0f} {m.get('SQ_INSTS_LDS', 0) / w:7.0f} "
          f"{2 * m.get('FETCH_SIZE', 0) / 1024:8.1f} {m.get('WRITE_SIZE', 0) / 1024:8.1f}")
