#!/usr/bin/env python3
"""Hash of the bf16 Generator's output on fixed synthetic weights and mel (B=5, T=200: every pair kernel walks
several tiles), for build-vs-build bit-identity checks (MT_LIB selects the library). Usage: python tools/gen_hash.py"""
import hashlib
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "matcha-tts_amd"))
sys.path.insert(0, os.path.join(HERE, "tests"))
import torch  # noqa: E402

if os.environ.get("MT_LIB"):
    import matcha_hip._lib as _L  # noqa: E402
    _L.LIB_PATH = os.environ["MT_LIB"]
from conftest import make_generator  # noqa: E402
from matcha_hip import synthetic  # noqa: E402

gen = make_generator("bf16")
sd = synthetic.make_state_dict([(k, tuple(v.shape)) for k, v in gen.state_dict().items()], 23)
gen.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
gen = gen.cuda().eval()
gen.remove_weight_norm()
mel = (torch.randn(5, 80, 200, generator=torch.Generator().manual_seed(9)) * 2 - 5).cuda()
with torch.inference_mode():
    a = gen(mel).float().cpu()
print("gen_hash", hashlib.sha256(a.numpy().tobytes()).hexdigest()[:16], float(a.abs().max()))
