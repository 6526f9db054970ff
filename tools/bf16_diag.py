#!/usr/bin/env python3
"""bf16 estimator error by block (debug taps, mt_decoder_set_taps) at the bench shape, for each decoder path:
vconv mode 1 (default), 2 (block 2's GroupNorm as a separate pass), 0 (generic conv kernel everywhere), and fp32.
Usage: python tools/bf16_diag.py [B] [T]"""
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "matcha-tts_amd"))
sys.path.insert(0, os.path.join(HERE, "tests"))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from conftest import make_decoder, rel_rms  # noqa: E402
from matcha_hip import synthetic  # noqa: E402
from oracle import matcha_oracle as O  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
T = int(sys.argv[2]) if len(sys.argv) > 2 else 728
dev = "cuda"
TAPS = ("down0_res", "down0_tb", "mid1_tb", "up0_out", "up1_tb")

rs = np.random.RandomState(B)
lens = np.clip(np.round(rs.normal(566, 150, B)), 96, T).astype(np.int64)
lens[0] = T
gen = torch.Generator().manual_seed(B)
x, mu = torch.randn(B, 80, T, generator=gen) * 0.667, torch.randn(B, 80, T, generator=gen)
mask = (torch.arange(T)[None] < torch.from_numpy(lens)[:, None]).float()[:, None]
mu = mu * mask
ref = {}
d0 = make_decoder(160, "fp32")
sd = {k: torch.from_numpy(v) for k, v in synthetic.make_state_dict(
    [(k, tuple(v.shape)) for k, v in d0.state_dict().items()], 5).items()}
with torch.inference_mode():
    ref_out = O.decoder_forward(sd, x, mask, mu, torch.full((B,), 0.3), taps=ref)


def mk(t):
    m = mask if mask.shape[-1] == t.shape[-1] else mask[:, :, ::2]
    return t * m


for prec, mode in (("bf16", 1), ("bf16", 2), ("bf16", 0), ("fp32", None)):
    dec = make_decoder(160, prec)
    dec.load_state_dict(sd)
    dec = dec.to(dev).eval()
    eng = dec.engine()
    if mode is not None:
        eng.set_vconv(mode)
    out, taps = eng.step_taps(dec.packed(dev), x.to(dev), mu.to(dev), mask.to(dev), None, 0.3)
    errs = {k: rel_rms(mk(taps[k].cpu()), mk(ref[k])) for k in TAPS}
    errs["out"] = rel_rms(out.cpu(), ref_out)
    print(f"{prec} vconv={mode}: " + ", ".join(f"{k} {v:.2e}" for k, v in errs.items()), flush=True)
