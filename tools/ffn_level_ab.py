#!/usr/bin/env python3
"""In-process A/B of the bf16 CFM decoder solve (10 Euler steps): mt_ffn on every level (MT_FFN_MIN = 0) against the
default frame threshold (level-1 blocks below it run FF1 + FF2 on mt_vconv). Usage: python tools/ffn_level_ab.py [B] [T]"""
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "matcha-tts_amd"))
sys.path.insert(0, os.path.join(HERE, "tests"))
import torch  # noqa: E402

from conftest import make_decoder  # noqa: E402
from matcha_hip import runtime as rt  # noqa: E402
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
mu = torch.randn(B, 80, T, generator=g).cuda()
lens = torch.randint(T // 3, T, (B,), generator=g)
lens[0] = T
mask = (torch.arange(T)[None] < lens[:, None]).float()[:, None].cuda()
mu = mu * mask
z = torch.randn(B, 80, T, generator=g).cuda()
default = rt.set_ffn_min_frames(16384)
rt.set_ffn_min_frames(default)
modes = {"default": default, "all-levels": 0}
res = {k: [] for k in modes}
outs = {}
for r in range(6):
    for k, v in modes.items():
        rt.set_ffn_min_frames(v)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        outs[k] = eng.solve(packed, z, 0.667, mu, mask, None, 10, "euler")
        torch.cuda.synchronize()
        if r > 0:
            res[k].append((time.perf_counter() - t0) * 1e3)
rt.set_ffn_min_frames(default)
for k in modes:
    v = sorted(res[k])
    print(f"decoder solve B={B} T={T} ffn {k}: median {v[len(v)//2]:.3f} ms min {v[0]:.3f} ms", flush=True)
print("bit-identical:", torch.equal(outs["default"], outs["all-levels"]))
