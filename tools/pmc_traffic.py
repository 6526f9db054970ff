#!/usr/bin/env python3
"""HBM traffic per launch of one kernel from two rocprofv3 counter passes (FETCH_SIZE, WRITE_SIZE).

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the bytes of wide
coalesced reads, so it is doubled; WRITE_SIZE is exact for 16-B stores. Both are in KiB.
Usage: python tools/pmc_traffic.py FETCH_CSV WRITE_CSV KERNEL_REGEX OUT_JSON "command"
Per kernel name, only the launches with that kernel's largest grid are used (the bench workload, not the
denoiser's bias-spectrum run on a 1 x 80 x 88 zero mel); the per-launch figure averages over all of them, so a
family of kernels (vconv + vpair) is weighted by its launch mix."""
import csv
import hashlib
import json
import os
import re
import sys

# what decides the family's HBM passes: its kernels' sources, every header they compile against (mt_common.h's
# epilogue helpers, mt_ragged.h's tile walk, ...), the Makefile's per-file flags and the path knobs (bench.py attaches
# the traffic only to a run whose own family key matches)
FAMILY_SOURCES = ("mt_rbconv.hip", "mt_vpair.hip", "mt_vpair32.hip", "mt_vpair128.hip", "mt_vconv.hip",
                  "mt_vocoder.hip")
FAMILY_KNOBS = ("MT_RBCONV", "MT_ACTIN", "MT_VPAIRK", "MT_VPAIR3", "MT_XCD_TILES")


def family_key(root):
    h = hashlib.sha1()
    csrc = os.path.join(root, "matcha-tts_amd", "csrc")
    headers = sorted(f for f in os.listdir(csrc) if f.endswith(".h"))
    for f in list(FAMILY_SOURCES) + headers:
        with open(os.path.join(csrc, f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    with open(os.path.join(root, "matcha-tts_amd", "Makefile"), "rb") as fh:
        h.update(fh.read())
    for k in FAMILY_KNOBS:
        h.update(f"{k}={os.environ.get(k, '')};".encode())
    return h.hexdigest()[:16]


def per_launch(path, sub, counter):
    rows = [r for r in csv.DictReader(open(path)) if re.search(sub, r["Kernel_Name"]) and r["Counter_Name"] == counter]
    gmax = {}
    for r in rows:
        gmax[r["Kernel_Name"]] = max(gmax.get(r["Kernel_Name"], 0), int(r["Grid_Size"]))
    keep = [r for r in rows if int(r["Grid_Size"]) == gmax[r["Kernel_Name"]]]
    vals = [float(r["Counter_Value"]) for r in keep]
    names = sorted({r["Kernel_Name"][:60] for r in keep})
    return sum(vals) / len(vals), len(vals), sorted(set(gmax.values())), names


if __name__ == "__main__":
    fetch, nf, grid, name = per_launch(sys.argv[1], sys.argv[3], "FETCH_SIZE")
    write, nw, _, _ = per_launch(sys.argv[2], sys.argv[3], "WRITE_SIZE")
    out = {"kernels": name, "grid_sizes": grid, "launches_fetch_pass": nf, "launches_write_pass": nw,
           "FETCH_SIZE_KiB": fetch, "WRITE_SIZE_KiB": write,
           "hbm_bytes_per_launch": int(round((2 * fetch + write) * 1024)),
           "correction": "2 x FETCH_SIZE (gfx950 reports half of wide coalesced reads) + WRITE_SIZE, KiB -> B",
           "command": sys.argv[5],
           "family_key": family_key(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))}
    json.dump(out, open(sys.argv[4], "w"), indent=1)
    print(json.dumps(out))
