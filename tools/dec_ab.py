#!/usr/bin/env python3
"""In-process A/B of the bf16 CFM decoder (10-step Euler solve): ResnetBlock / k=3 convs on mt_vconv
vs the generic conv kernel (interleaved rounds, one process, random data, full-length rows except one).
Usage: python tools/dec_ab.py [B] [T] [rounds] [modes, e.g. 10 or 1]"""
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "matcha-tts_amd"))
sys.path.insert(0, os.path.join(HERE, "tests"))
import torch  # noqa: E402

from conftest import make_decoder  # noqa: E402
from matcha_hip import synthetic  # noqa: E402
if os.environ.get("MT_LIB"):  # timing experiments: another build of the library
    import matcha_hip._lib as _L  # noqa: E402
    _L.LIB_PATH = os.environ["MT_LIB"]

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
T = int(sys.argv[2]) if len(sys.argv) > 2 else 728
R = int(sys.argv[3]) if len(sys.argv) > 3 else 3
dec = make_decoder(160, "bf16")
sd = synthetic.make_state_dict([(k, tuple(v.shape)) for k, v in dec.state_dict().items()], 7)
dec.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
dec = dec.cuda().eval()
eng = dec.engine()
packed = dec.packed(torch.device("cuda", 0))
g = torch.Generator().manual_seed(0)
mu = torch.randn(B, 80, T, generator=g).cuda()
# ragged like the bench's batch: one full-length row, the rest padded (RAGGED=0: all full but one)
if os.environ.get("RAGGED", "1") == "1":
    lens = torch.randint(T // 3, T, (B,), generator=g)
    lens[0] = T
else:
    lens = torch.full((B,), T)
    lens[-1] = T * 2 // 3
mask = (torch.arange(T)[None] < lens[:, None]).float()[:, None].cuda()
mu = mu * mask
z = torch.randn(B, 80, T, generator=g).cuda()
MODES = tuple(int(c) for c in sys.argv[4]) if len(sys.argv) > 4 else (1, 0)
res = {m: [] for m in MODES}
outs = {}
for r in range(R + 1):
    for m in MODES:
        eng.set_vconv(m)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        outs[m] = eng.solve(packed, z, 0.667, mu, mask, None, 10, "euler")
        torch.cuda.synchronize()
        if r > 0:
            res[m].append((time.perf_counter() - t0) * 1e3)
for m in MODES:
    v = sorted(res[m])
    print(f"decoder solve B={B} T={T} vconv={m}: median {v[len(v)//2]:.2f} ms min {v[0]:.2f} ms", flush=True)
if len(outs) == 2:
    d = (outs[1] - outs[0]).float()
    print(f"rel-RMS(vconv vs generic) = {(d.pow(2).mean() / outs[0].float().pow(2).mean()).sqrt().item():.3e}")
