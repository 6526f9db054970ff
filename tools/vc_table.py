"""Per-launch TF/s of the vconv (and fused stage) kernels of the first vconv-on vocoder call in a trace."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
seq = [(r['Kernel_Name'], (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6) for r in rows
       if 'vconv_kernel' in r['Kernel_Name']]
ks, ds = [3, 7, 11], [1, 3, 5]
Ltot = 32 * 728
i, tot = 0, {}
for st, (C, L) in enumerate([(256, 8 * Ltot), (128, 64 * Ltot)]):
    for k in ks:
        for d in ds:
            for half in (0, 1):
                n, t = seq[i]
                i += 1
                fl = 2 * C * C * k * L
                tot[st] = tot.get(st, 0) + t
                print(f"stage{st + 1} C={C} k={k:2d} d={d if half == 0 else 1} {'conv1' if half == 0 else 'conv2'} "
                      f"{t:.3f} ms {fl / t / 1e9:7.1f} TF/s  {n[:28]}")
for st, t in tot.items():
    print(f"stage{st + 1} vconv total {t:.2f} ms")
for r in rows:
    pass
