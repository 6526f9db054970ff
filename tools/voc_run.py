#!/usr/bin/env python3
"""Vocoder-only driver for counter passes: HiFi-GAN v1 bf16 on B x T synthetic mel, R runs."""
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

B = int(os.environ.get("VB", "32"))
T = int(os.environ.get("VT", "728"))
R = int(os.environ.get("VR", "3"))
g = Generator(AttrDict(v1), precision="bf16")
sd = synthetic.make_state_dict([(k, tuple(v.shape)) for k, v in g.state_dict().items()], 7)
g.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
g = g.cuda().eval()
g.remove_weight_norm()
mel = (torch.randn(B, 80, T) * 2 - 5).cuda()
for _ in range(R):
    wav = g(mel)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(R):
    wav = g(mel)
torch.cuda.synchronize()
print(f"vocoder B={B} T={T}: {(time.perf_counter() - t0) / R * 1e3:.2f} ms", flush=True)
