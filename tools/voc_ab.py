#!/usr/bin/env python3
"""In-process A/B of the bf16 vocoder (interleaved rounds, one process, random-data mel). MODES: digits of
vconv modes (2: per-layer vconv incl. the 64-channel stage, 1: that stage on the fused rbfuse kernel, 0: generic);
PAIR=1 adds "p" = mode 2 with the 64-channel stage's ResBlock pairs fused (mt_vpair).
Usage: [MODES=210] [PAIR=1] python tools/voc_ab.py [B] [T] [rounds]"""
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "matcha-tts_amd"))
import torch  # noqa: E402

from hifigan.config import v1  # noqa: E402
from hifigan.env import AttrDict  # noqa: E402
from hifigan.models import Generator  # noqa: E402
from matcha_hip import synthetic  # noqa: E402
if os.environ.get("MT_LIB"):  # timing experiments: another build of the library
    import matcha_hip._lib as _L  # noqa: E402
    _L.LIB_PATH = os.environ["MT_LIB"]
MODES = tuple(int(c) for c in os.environ.get("MODES", "210")) + (("p",) if os.environ.get("PAIR") == "1" else ())

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
T = int(sys.argv[2]) if len(sys.argv) > 2 else 728
R = int(sys.argv[3]) if len(sys.argv) > 3 else 3
g = Generator(AttrDict(v1), precision="bf16")
sd = synthetic.make_state_dict([(k, tuple(v.shape)) for k, v in g.state_dict().items()], 7)
g.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
g = g.cuda().eval()
g.remove_weight_norm()
mel = (torch.randn(B, 80, T) * 2 - 5).cuda()
eng = g.engine()
res = {m: [] for m in MODES}
for r in range(R + 1):
    for on in MODES:
        eng.set_vconv(2 if on == "p" else on)
        eng.set_pair(on == "p")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        wav = g(mel)
        torch.cuda.synchronize()
        if r > 0:
            res[on].append((time.perf_counter() - t0) * 1e3)
for on in MODES:
    v = sorted(res[on])
    if not v:
        continue
    print(f"vocoder B={B} T={T} vconv={on}: median {v[len(v)//2]:.2f} ms min {v[0]:.2f} ms", flush=True)
