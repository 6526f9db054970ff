#!/usr/bin/env python3
"""Phase timing of every mt_vconv launch of one bf16 CFM solve (B, T as the bench), from the -DVCONV_TS build
(matcha-tts_amd/libmatcha_hip_ts.so): per workgroup s_memrealtime (100 MHz) at entry, after the prologue's first
data wait, at the end of its first tile's K loop, and after its last stores landed. Per launch class (epilogue,
tile, 1x1, taps, M, cin, L): launch span (first entry .. last end), dispatch spread (entry of the last workgroup
- first), prologue (median entry -> data ready), first tile K loop, tail (K-loop end -> end: epilogue + later
tiles + store drain) and the gap to the next launch's first entry.
Usage: MT_LIB=matcha-tts_amd/libmatcha_hip_ts.so python tools/vconv_ts.py [B] [T]"""
import ctypes
import os
import sys
from collections import defaultdict

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "matcha-tts_amd"))
sys.path.insert(0, os.path.join(HERE, "tests"))
import torch  # noqa: E402

import matcha_hip._lib as _L  # noqa: E402
_L.LIB_PATH = os.environ.get("MT_LIB", os.path.join(HERE, "matcha-tts_amd", "libmatcha_hip_ts.so"))
from conftest import make_decoder  # noqa: E402
from matcha_hip import synthetic  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
T = int(sys.argv[2]) if len(sys.argv) > 2 else 728
dec = make_decoder(160, "bf16")
sd = synthetic.make_state_dict([(k, tuple(v.shape)) for k, v in dec.state_dict().items()], 7)
dec.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
dec = dec.cuda().eval()
eng = dec.engine()
packed = dec.packed(torch.device("cuda", 0))
g = torch.Generator().manual_seed(0)
lens = torch.randint(T // 3, T - 2, (B,), generator=g)
lens[0] = T - 2  # every row padded: the bench's query-independent attention path
mask = (torch.arange(T)[None] < lens[:, None]).float()[:, None].cuda()
mu = torch.randn(B, 80, T, generator=g).cuda() * mask
z = torch.randn(B, 80, T, generator=g).cuda()
L = _L.lib()
f = L.mt_vconv_ts_dump
f.restype = ctypes.c_int
f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
MAXS = 4096
ts = np.zeros(MAXS * 256 * 4, np.uint64)
meta = np.zeros(MAXS * 11, np.int32)
eng.set_graphs(0)  # direct launches: each one assigns its own timestamp slot
mv = int(lens.max())  # synthesize's y_max: the query-independent attention, as in the bench
for _ in range(2):  # warm-up (packs)
    eng.solve(packed, z, 0.667, mu, mask, None, 10, "euler", max_valid=mv)
torch.cuda.synchronize()
f(ts.ctypes.data, meta.ctypes.data, MAXS)  # discard
eng.solve(packed, z, 0.667, mu, mask, None, 10, "euler", max_valid=mv)
torch.cuda.synchronize()
n = f(ts.ctypes.data, meta.ctypes.data, MAXS)
ts = ts[:n * 1024].reshape(n, 256, 4).astype(np.int64)
meta = meta[:n * 11].reshape(n, 11)
rows = []
for i in range(n):
    G = int(meta[i, 5])
    t = ts[i, :G]
    t0, t1, t2, t3 = t[:, 0], t[:, 1], t[:, 2], t[:, 3]
    span = t3.max() - t0.min()
    nxt = ts[i + 1, :int(meta[i + 1, 5]), 0].min() - t3.max() if i + 1 < n else 0
    rows.append((tuple(int(v) for v in meta[i]), span, t0.max() - t0.min(), np.median(t1 - t0),
                 np.median(t2 - t1), np.median(t3 - t2), nxt))
agg = defaultdict(list)
for r in rows:
    agg[r[0]].append(r[1:])
print(f"{n} vconv launches in one B={B} T={T} solve (times in us; 100 MHz clock)")
print(f"{'ef':>6s} {'BM':>4s} {'BN':>4s} {'k1':>2s} {'tiles':>6s} {'G':>4s} {'taps':>4s} {'M':>5s} {'cin':>5s} {'L':>6s} "
      f"{'n':>4s} {'span':>7s} {'spread':>7s} {'prolog':>7s} {'kloop1':>7s} {'tail':>7s} {'gap':>7s} {'sum':>8s}")
tot = 0.0
for k, v in sorted(agg.items(), key=lambda kv: -sum(x[0] for x in kv[1])):
    a = np.array(v, dtype=np.float64) / 100.0  # 10 ns ticks -> us
    m = a.mean(axis=0)
    tot += a[:, 0].sum()
    ef, BM, BN, k1, tiles, G, taps, M, cin, Bq, Lq = k
    print(f"{ef:6d} {BM:4d} {BN:4d} {k1:2d} {tiles:6d} {G:4d} {taps:4d} {M:5d} {cin:5d} {Lq:6d} {len(v):4d} "
          f"{m[0]:7.1f} {m[1]:7.1f} {m[2]:7.1f} {m[3]:7.1f} {m[4]:7.1f} {m[5]:7.1f} {a[:, 0].sum():8.0f}")
print(f"total vconv span {tot / 1000:.2f} ms")
