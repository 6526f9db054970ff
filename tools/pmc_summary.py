#!/usr/bin/env python3
"""Summarise tools/pmc.sh passes: per kernel (and launch shape), mean counters per dispatch.
Usage: python tools/pmc_summary.py gpurun_out/TAG [kernel-substring]"""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
agg = defaultdict(lambda: defaultdict(list))  # (kernel, grid) -> counter -> values
dur = defaultdict(list)
for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = (r["Kernel_Name"], int(r["Grid_Size"]))
        if flt and flt not in k[0]:
            continue
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if r["Counter_Name"] in ("SQ_WAVES", "FETCH_SIZE"):
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
for k, cs in sorted(agg.items(), key=lambda kv: -sum(dur[kv[0]]) if dur[kv[0]] else 0):
    name = k[0][:90]
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    print(f"{name} grid={k[1]} n={len(next(iter(cs.values())))} us/launch(pmc)={sum(dur[k]) / max(1, len(dur[k])):.1f}")
    wc = m.get("SQ_WAVE_CYCLES", 0)
    line = []
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if c in m:
                line.append(f"{c[3:]}={m[c] / wc:.2f}")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
        pass
    if "SQ_BUSY_CYCLES" in m and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
        line.append(f"MFMA_BUSY/BUSY={m['SQ_VALU_MFMA_BUSY_CYCLES'] / max(1, m['SQ_BUSY_CYCLES']):.3f}")
    if "SQ_LDS_IDX_ACTIVE" in m:
        line.append(f"LDS_conflict/active={m.get('SQ_LDS_BANK_CONFLICT', 0) / max(1, m['SQ_LDS_IDX_ACTIVE']):.3f}")
    if "FETCH_SIZE" in m:
        line.append(f"FETCH_KB(x2)={2 * m['FETCH_SIZE']:.0f}")
    if "WRITE_SIZE" in m:
        line.append(f"WRITE_KB={m['WRITE_SIZE']:.0f}")
    print("   ", " ".join(line))
    print("   ", " ".join(f"{c}={v:.4g}" for c, v in sorted(m.items())))
