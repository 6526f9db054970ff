"""In-process A/B of conv tile variants on the decoder's GEMM shapes (B=32, T=728; GPU only).
Usage: python tools/ab_gemm.py [variants]"""
import math, sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "matcha-tts_amd"))
import torch
from matcha_hip import runtime as rt

dev = torch.device("cuda", 0)
T = 728
shapes = [  # name, cin, cout, k, frames
    ("outproj T/2", 128, 256, 1, 32 * T // 2),
    ("ff2 T/2", 1024, 256, 1, 32 * T // 2),
    ("ff1 T", 256, 1024, 1, 32 * T),
    ("qkv T", 256, 384, 1, 32 * T),
    ("conv3 T", 256, 256, 3, 32 * T),
    ("conv3 T/2", 256, 256, 3, 32 * T // 2),
]
variants = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else [-1, 1, 2, 5, 6, 7, 8, 9, 11, 12, 13, 14, 15]
for name, cin, cout, k, L in shapes:
    g = torch.Generator().manual_seed(0)
    x = torch.randn(32, L // 32, cin, generator=g).to(dev).bfloat16()
    W = (torch.randn(cout, cin, k, generator=g) / math.sqrt(cin * k)).to(dev)
    b = torch.zeros(cout, device=dev)
    y = torch.empty(32, L // 32, cout, dtype=torch.bfloat16, device=dev)
    fl = 2.0 * cout * cin * k * L
    ref = None
    line = []
    for v in variants:
        if k > 1 and v in (11, 13, 14, 15, 6):
            continue
        try:
            nb = rt.lib().mt_op_conv1d_workspace_bytes(1, cin, cout, k, 1, 0)
            ws = torch.empty(nb, dtype=torch.uint8, device=dev)
            out = rt.op_conv1d(x, W, b, 1, (k - 1) // 2, 1, False, 0.1, "bf16", v, out=y, ws=ws).float()
        except Exception as e:  # variant cannot serve this shape
            continue
        if ref is None:
            ref = out.clone()
        err = (out - ref).abs().max().item()
        ts = []
        for r in range(5):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                rt.op_conv1d(x, W, b, 1, (k - 1) // 2, 1, False, 0.1, "bf16", v + 0x1000, out=y, ws=ws)
            e.record(); torch.cuda.synchronize()
            ts.append(s.elapsed_time(e) / 5)
        t = min(ts)
        line.append(f"v{v}:{t*1e3:.0f}us/{fl/t/1e9:.0f}TF{'!' if err > 0.05 else ''}")
    print(f"{name:12s} " + " ".join(line), flush=True)
