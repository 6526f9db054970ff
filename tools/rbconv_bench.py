#!/usr/bin/env python3
"""Op-level timing of the HiFi-GAN stage-1/2 ResBlock convs (B=32, T=728 mel frames as one long utterance per
shape), mt_rbconv (compile-time K-loop schedule) against the generic mt_vconv kernel, interleaved in one process,
weights packed once. Usage: python tools/rbconv_bench.py [rounds] [B]"""
import math
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "matcha-tts_amd"))
import torch  # noqa: E402

if os.environ.get("MT_LIB"):  # timing experiments: another build of the library
    import matcha_hip._lib as _L  # noqa: E402
    _L.LIB_PATH = os.environ["MT_LIB"]

from matcha_hip import runtime as rt  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 5
B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
dev = torch.device("cuda", 0)
ACT, RD, RADD = 8, 1 | 16, 1 | 2 | 4 | 16
shapes = [  # name, C, k, d, frames, ef
    ("s1 k3 d1 conv1", 256, 3, 1, B * 8 * 728, ACT),
    ("s1 k7 d3 conv1", 256, 7, 3, B * 8 * 728, ACT),
    ("s1 k11 d5 conv1", 256, 11, 5, B * 8 * 728, ACT),
    ("s1 k3 conv2", 256, 3, 1, B * 8 * 728, RD),
    ("s1 k11 conv2 last", 256, 11, 1, B * 8 * 728, RADD),
    ("s2 k7 d3 conv1", 128, 7, 3, B * 64 * 728, ACT),
    ("s2 k11 d5 conv1", 128, 11, 5, B * 64 * 728, ACT),
    ("s2 k7 conv2", 128, 7, 1, B * 64 * 728, RD),
    ("s2 k11 conv2 last", 128, 11, 1, B * 64 * 728, RADD),
]
tot = {True: 0.0, False: 0.0}
for name, C, k, d, L, ef in shapes:
    g = torch.Generator().manual_seed(0)
    x = torch.randn(1, L, C, generator=g).to(dev).bfloat16()
    W = (torch.randn(C, C, k, generator=g) / math.sqrt(C * k)).to(dev)
    b = torch.zeros(C, device=dev)
    resid = torch.randn(1, L, C, generator=g).to(dev).bfloat16()
    y = torch.randn(1, L, C, generator=g).to(dev).bfloat16()
    y2 = torch.empty_like(y)
    nb = rt.lib().mt_op_vconv_workspace_bytes(C, C, k)
    ws = torch.empty(nb, dtype=torch.uint8, device=dev)
    rt.op_vconv(x, W, b, d, ef, resid if ef & 1 else None, y=y, y2=y2, ws=ws, pack=True, div=3.0)
    res = {True: [], False: []}
    for r in range(R):
        for v in (True, False):
            prev = rt.set_rbconv(v)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                rt.op_vconv(x, W, b, d, ef, resid if ef & 1 else None, y=y, y2=y2, ws=ws, pack=False, div=3.0)
            e.record()
            torch.cuda.synchronize()
            rt.set_rbconv(prev)
            res[v].append(s.elapsed_time(e) / 5)
    fl = 2.0 * C * C * k * L
    line = f"{name:18s}"
    for v in (True, False):
        ts = sorted(res[v])
        tot[v] += ts[len(ts) // 2]
        line += f" | {'rb' if v else 'vc'} {ts[len(ts) // 2]:7.3f} ms {fl / ts[len(ts) // 2] / 1e9:7.1f} TF/s"
    print(line, flush=True)
print(f"total rb {tot[True]:.3f} ms  vc {tot[False]:.3f} ms  ratio {tot[True] / tot[False]:.3f}", flush=True)
