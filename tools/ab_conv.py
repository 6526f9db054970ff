"""In-process A/B timing of conv tile variants on the dominant layer shapes (GPU only)."""
import math, sys, os, json
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "matcha-tts_amd"))
import torch
from matcha_hip import runtime as rt

dev = torch.device("cuda", 0)
shapes = [  # (name, C, k, d, frames)
    ("s2_k11d5", 128, 11, 5, 32 * 64 * 728),
    ("s2_k3d1", 128, 3, 1, 32 * 64 * 728),
    ("s1_k7d3", 256, 7, 3, 32 * 8 * 728),
]
variants = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else list(range(11))
reps, rounds = 5, 3
res = {}
for name, C, k, d, L in shapes:
    g = torch.Generator().manual_seed(0)
    x = torch.randn(1, L, C, generator=g).to(dev).bfloat16()
    W = (torch.randn(C, C, k, generator=g) / math.sqrt(C * k)).to(dev)
    b = torch.zeros(C, device=dev)
    y = torch.empty(1, L, C, dtype=torch.bfloat16, device=dev)
    ref = rt.op_conv1d(x, W, b, 1, d * (k - 1) // 2, d, False, 0.1, "bf16", -1).float()
    flops = 2.0 * C * C * k * L
    for v in variants:
        out = rt.op_conv1d(x, W, b, 1, d * (k - 1) // 2, d, False, 0.1, "bf16", v, out=y)
        err = (out.float() - ref).abs().max().item()
        res.setdefault((name, v), {"err": err, "ms": []})
    for r in range(rounds):
        for v in variants:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(reps):
                rt.op_conv1d(x, W, b, 1, d * (k - 1) // 2, d, False, 0.1, "bf16", v, out=y)
            e.record(); torch.cuda.synchronize()
            res[(name, v)]["ms"].append(s.elapsed_time(e) / reps)
    for v in variants:
        ms = sorted(res[(name, v)]["ms"])
        print(f"{name:10s} variant {v}: median {ms[len(ms)//2]:.3f} ms  min {ms[0]:.3f}  "
              f"{flops / (ms[0] * 1e-3) / 1e12:7.1f} TF/s  maxerr {res[(name, v)]['err']:.2e}", flush=True)
