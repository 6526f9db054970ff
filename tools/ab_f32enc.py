"""In-process A/B of conv tile variants in fp32 on the text encoder's shapes (B=32, Tx=242). GPU only.
Usage: python tools/ab_f32enc.py [variants]"""
import math, sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "matcha-tts_amd"))
import torch
from matcha_hip import runtime as rt

dev = torch.device("cuda", 0)
shapes = [("ffn1", 192, 768, 3), ("ffn2", 768, 192, 3), ("pre_k5", 192, 192, 5), ("qkv", 192, 576, 1), ("dp1", 192, 256, 3)]
variants = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else [-1] + list(range(16))
B, T, reps = 32, 242, 5
for name, cin, cout, k in shapes:
    g = torch.Generator().manual_seed(0)
    x = torch.randn(B, T, cin, generator=g).to(dev)
    W = (torch.randn(cout, cin, k, generator=g) / math.sqrt(cin * k)).to(dev)
    b = torch.zeros(cout, device=dev)
    y = torch.empty(B, T, cout, device=dev)
    ref = rt.op_conv1d(x, W, b, 1, k // 2, 1, False, 0.1, "fp32", -1).clone()
    flops = 2.0 * cin * cout * k * B * T
    for v in variants:
        try:
            out = rt.op_conv1d(x, W, b, 1, k // 2, 1, False, 0.1, "fp32", v, out=y)
        except Exception as e:
            print(f"{name} variant {v}: {e}")
            continue
        err = (out - ref).abs().max().item()
        ts = []
        for r in range(3):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(reps):
                rt.op_conv1d(x, W, b, 1, k // 2, 1, False, 0.1, "fp32", v, out=y)
            e.record(); torch.cuda.synchronize()
            ts.append(s.elapsed_time(e) / reps)
        t = min(ts)
        print(f"{name:7s} variant {v:3d}: {t * 1e3:8.1f} us {flops / (t * 1e-3) / 1e12:7.1f} TF/s maxerr {err:.1e}", flush=True)
