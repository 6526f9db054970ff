#!/usr/bin/env python3
"""MAS timing: mt_maximum_path on a training-shaped batch (B utterances, t_x tokens, 3 frames/token
ragged like the bench) vs the oracle restatement of the reference's Python DP on one utterance (CPU).
Usage: python tools/mas_bench.py [B] [Tx]"""
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "matcha-tts_amd"))
sys.path.insert(0, HERE)
import torch  # noqa: E402

from matcha_hip import runtime as rt  # noqa: E402
from oracle import matcha_oracle as O  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
TX = int(sys.argv[2]) if len(sys.argv) > 2 else 250
g = torch.Generator().manual_seed(0)
t_xs = torch.randint(TX // 3, TX + 1, (B,), generator=g)
t_xs[0] = TX
t_ys = t_xs * 3
Tx, Ty = int(t_xs.max()), int(t_ys.max())
neg = torch.randn(B, Tx, Ty, generator=g) * 10 - 80
xm = (torch.arange(Tx)[None] < t_xs[:, None]).float()
ym = (torch.arange(Ty)[None] < t_ys[:, None]).float()
mask = xm[:, :, None] * ym[:, None, :]
dn, dm = neg.cuda(), mask.cuda()
rt.maximum_path(dn, dm)
torch.cuda.synchronize()
ts = []
for _ in range(5):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    rt.maximum_path(dn, dm)
    e.record()
    torch.cuda.synchronize()
    ts.append(s.elapsed_time(e))
t0 = time.perf_counter()
O.maximum_path(neg[:1], mask[:1])
cpu = time.perf_counter() - t0
print(f"MAS B={B} Tx={Tx} Ty={Ty}: GPU {sorted(ts)[2]:.3f} ms per batch; "
      f"oracle (reference's Python DP restated) {cpu * 1e3:.0f} ms for ONE utterance ({t_xs[0]}x{t_ys[0]})",
      flush=True)
