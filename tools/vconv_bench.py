#!/usr/bin/env python3
"""Op-level timing of mt_vconv on the HiFi-GAN v1 stage-1/2 shapes (B=32, T=728 mel frames), weights
packed once, interleaved rounds in one process. Usage: python tools/vconv_bench.py [rounds]"""
import math
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "matcha-tts_amd"))
import torch  # noqa: E402

from matcha_hip import runtime as rt  # noqa: E402
if os.environ.get("MT_LIB"):  # timing experiments: another build of the library
    import matcha_hip._lib as _L  # noqa: E402
    _L.LIB_PATH = os.environ["MT_LIB"]

R = int(sys.argv[1]) if len(sys.argv) > 1 else 5
VARIANTS = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0]
dev = torch.device("cuda", 0)
shapes = [  # name, C, k, d, frames, ef
    ("s2 k3 conv1", 128, 3, 1, 32 * 64 * 728, 8),
    ("s2 k11 conv1", 128, 11, 5, 32 * 64 * 728, 8),
    ("s2 k3 conv2", 128, 3, 1, 32 * 64 * 728, 1 | 16),
    ("s2 k11 conv2", 128, 11, 1, 32 * 64 * 728, 1 | 16),
    ("s1 k7 conv1", 256, 7, 3, 32 * 8 * 728, 8),
    ("s3 k11 conv1", 64, 11, 5, 32 * 128 * 728, 8),
    ("s3 k3 conv2", 64, 3, 1, 32 * 128 * 728, 1 | 16),
]
for name, C, k, d, L, ef in shapes:
    g = torch.Generator().manual_seed(0)
    x = torch.randn(1, L, C, generator=g).to(dev).bfloat16()
    W = (torch.randn(C, C, k, generator=g) / math.sqrt(C * k)).to(dev)
    b = torch.zeros(C, device=dev)
    resid = torch.randn(1, L, C, generator=g).to(dev).bfloat16()
    y = torch.empty(1, L, C, dtype=torch.bfloat16, device=dev)
    y2 = torch.empty_like(y)
    nb = rt.lib().mt_op_vconv_workspace_bytes(C, C, k)
    ws = torch.empty(nb, dtype=torch.uint8, device=dev)
    rt.op_vconv(x, W, b, d, ef, resid if ef & 1 else None, y=y, y2=y2, ws=ws, pack=True)
    res = {v: [] for v in VARIANTS}
    for r in range(R):
        for v in VARIANTS:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                rt.op_vconv(x, W, b, d, ef, resid if ef & 1 else None, y=y, y2=y2, ws=ws, pack=False)
            e.record()
            torch.cuda.synchronize()
            res[v].append(s.elapsed_time(e) / 5)
    fl = 2.0 * C * C * k * L
    by = 2.0 * L * C * (2 + (1 if ef & 1 else 0) + (1 if ef & 16 else 0))
    for v in VARIANTS:
        ts = sorted(res[v])
        print(f"{name:14s} v{v} {ts[len(ts)//2]:.3f} ms  {fl / ts[0] / 1e9:7.1f} TF/s  {by / ts[0] / 1e6:6.0f} GB/s",
              flush=True)
