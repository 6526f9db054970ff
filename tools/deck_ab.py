#!/usr/bin/env python3
"""In-process A/B of the decoder kernel variants (mt_decoder_set_kernels masks, bit-identical): the bf16 CFM solve
(10-step Euler, graph path) at B x T, ragged like the bench (the longest utterance T - 4 frames, so the
query-independent attention runs at both levels), interleaved rounds, median and min per mask; checks the outputs
are equal. Usage: python tools/deck_ab.py [B] [T] [rounds] [masks, e.g. 0,1]"""
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
R = int(sys.argv[3]) if len(sys.argv) > 3 else 5
MASKS = [int(c) for c in sys.argv[4].split(",")] if len(sys.argv) > 4 else [0, 1]
dec = make_decoder(160, "bf16")
sd = synthetic.make_state_dict([(k, tuple(v.shape)) for k, v in dec.state_dict().items()], 7)
dec.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
dec = dec.cuda().eval()
eng = dec.engine()
packed = dec.packed(torch.device("cuda", 0))
g = torch.Generator().manual_seed(0)
lens = torch.randint(T // 3, T - 4, (B,), generator=g)
lens[0] = T - 4
mask = (torch.arange(T)[None] < lens[:, None]).float()[:, None].cuda()
mu = torch.randn(B, 80, T, generator=g).cuda() * mask
z = torch.randn(B, 80, T, generator=g).cuda()
res = {m: [] for m in MASKS}
outs = {}
for r in range(R + 1):
    for m in MASKS:
        prev = rt.set_decoder_kernels(m)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        outs[m] = eng.solve(packed, z, 0.667, mu, mask, None, 10, "euler", max_valid=int(lens.max()))
        torch.cuda.synchronize()
        if r > 0:
            res[m].append((time.perf_counter() - t0) * 1e3)
        rt.set_decoder_kernels(prev)
for m in MASKS:
    v = sorted(res[m])
    print(f"decoder solve B={B} T={T} mask={m}: median {v[len(v) // 2]:.3f} ms min {v[0]:.3f} ms", flush=True)
print("outputs equal:", all(torch.equal(outs[m], outs[MASKS[0]]) for m in MASKS))
