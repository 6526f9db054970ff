"""Shared test fixtures.

* ``gpu`` marker: tests that need the MI355X; everything else runs on CPU.
* The product package lives in ``matcha-tts_amd/`` (drop-in ``model`` / ``hifigan``
  modules + ``matcha_hip`` runtime); the oracle in ``oracle/`` is test infrastructure.
* Golden vectors (tests/golden/*.npz) were produced by running the reference itself
  (tests/golden/make_golden.py); weights are regenerated from the committed recipe.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "matcha-tts_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (PKG, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

from matcha_hip import synthetic  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm) GPU and the built HIP library")


def pytest_collection_modifyitems(config, items):
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no ROCm GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


def golden(name: str):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def weights_from(g, prefix: str = ""):
    """Synthetic reference-keyed state dict of a golden fixture (recipe + seed + manifest)."""
    man = json.loads(str(g["manifest"]))
    sd = synthetic.make_state_dict([(k, tuple(s)) for k, s in man], int(g["seed"]))
    return {prefix + k: torch.from_numpy(v) for k, v in sd.items()}


def t(a, device="cpu"):
    return torch.from_numpy(np.asarray(a)).to(device)


ENC = dict(encoder_type="RoPE Encoder", n_feats=80, n_channels=192, filter_channels=768, n_heads=2,
           n_layers=6, kernel_size=3, p_dropout=0.1, prenet=True)
DEC = dict(channels=(256, 256), dropout=0.05, attention_head_dim=64, n_blocks=1, num_mid_blocks=2,
           num_heads=2, act_fn="snakebeta")
DP = dict(filter_channels_dp=256, kernel_size=3, p_dropout=0.1)
HP = dict(n_channels=192, n_layers=6, n_heads=2, kernel_size=3, dp_kernel_size=3)


def make_matcha(n_spks=1, precision="fp32"):
    from types import SimpleNamespace

    import model
    return model.MatchaTTS(178, n_spks, 64, SimpleNamespace(**ENC), SimpleNamespace(**DEC),
                           {"solver": "euler", "sigma_min": 1e-4}, SimpleNamespace(**DP), precision=precision)


def make_decoder(c_cond, precision="fp32"):
    import model
    return model.Decoder(in_channels=c_cond, out_channels=80, precision=precision, **DEC)


def make_generator(precision="fp32"):
    from hifigan.config import v1
    from hifigan.env import AttrDict
    from hifigan.models import Generator
    return Generator(AttrDict(v1), precision=precision)


def rel_rms(a: torch.Tensor, b: torch.Tensor) -> float:
    a, b = a.double(), b.double()
    return float(torch.sqrt(((a - b) ** 2).mean()) / torch.sqrt((b ** 2).mean()).clamp_min(1e-30))
