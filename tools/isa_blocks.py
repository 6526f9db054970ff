#!/usr/bin/env python3
"""Instruction mix per basic block of one kernel in a device assembly file (`hipcc --cuda-device-only -S`).

Counts MFMA, VALU (non-MFMA vector ALU), DS (LDS), VMEM (global / buffer, LDS-DMA included), SALU, waits and barriers
per block, and the issue-cycle estimate of each block from MI355X_MICROARCH.md's constants (VALU 4 cycles, an 8-cycle
transcendental, the MFMA's 8-cycle issue hold; 16x16x32 bf16 MFMA 16 cycles of matrix pipe). Used to count the VALU
per output element of the pair kernels before and after a change.
Usage: python tools/isa_blocks.py FILE.s KERNEL_SUBSTRING [--min N]"""
import re
import sys

TRANS = ("v_exp", "v_log", "v_rcp", "v_rsq", "v_sqrt", "v_sin", "v_cos")


def kind(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "ds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op == "s_waitcnt" or op.startswith("s_waitcnt"):
        return "wait"
    if op == "s_barrier":
        return "bar"
    if op.startswith("s_"):
        return "salu"
    return None


def main():
    path, name = sys.argv[1], sys.argv[2]
    mn = int(sys.argv[sys.argv.index("--min") + 1]) if "--min" in sys.argv else 1
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        if re.match(r"^_Z\S*:", l) and name in l.split(":")[0]:
            start = i
            break
    if start is None:
        sys.exit(f"kernel {name} not found")
    blocks, cur, label = [], None, lines[start].split(":")[0][-40:]
    cur = {"label": label, "n": {}, "trans": 0, "lines": 0}
    for l in lines[start + 1:]:
        if l.startswith("\t.end_amdhsa_kernel") or re.match(r"^\.Lfunc_end", l):
            break
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            blocks.append(cur)
            cur = {"label": m.group(1), "n": {}, "trans": 0, "lines": 0}
            continue
        t = l.strip().split()
        if not t or t[0].startswith((";", ".")):
            continue
        k = kind(t[0])
        if k is None:
            continue
        cur["n"][k] = cur["n"].get(k, 0) + 1
        cur["lines"] += 1
        if t[0].startswith(TRANS):
            cur["trans"] += 1
    blocks.append(cur)
    tot = {}
    print(f"{'block':>14s} {'mfma':>5s} {'valu':>5s} {'ds':>4s} {'vmem':>4s} {'salu':>4s} {'wait':>4s} {'bar':>3s}"
          f" {'vcyc':>6s} {'mcyc':>6s}")
    for b in blocks:
        n = b["n"]
        for k, v in n.items():
            tot[k] = tot.get(k, 0) + v
        if b["lines"] < mn:
            continue
        vcyc = 4 * n.get("valu", 0) + 4 * b["trans"] + 8 * n.get("mfma", 0)
        print(f"{b['label'][-14:]:>14s} {n.get('mfma', 0):5d} {n.get('valu', 0):5d} {n.get('ds', 0):4d} "
              f"{n.get('vmem', 0):4d} {n.get('salu', 0):4d} {n.get('wait', 0):4d} {n.get('bar', 0):3d} "
              f"{vcyc:6d} {16 * n.get('mfma', 0):6d}")
    print("total", tot)


if __name__ == "__main__":
    main()
