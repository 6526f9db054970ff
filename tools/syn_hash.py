#!/usr/bin/env python3
"""Hashes of the bench step's mel and denoised waveform (bf16 text->wav at B = 6 and 40: the decoder's convs on
one-round and multi-round grids, the ragged vocoder) with the CFM noise fixed, for build-vs-build bit-identity checks
(MT_LIB selects the library). Usage: python tools/syn_hash.py"""
import hashlib
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "matcha-tts_amd"))
sys.path.insert(0, HERE)
import torch  # noqa: E402

if os.environ.get("MT_LIB"):
    import matcha_hip._lib as _L  # noqa: E402
    _L.LIB_PATH = os.environ["MT_LIB"]
import bench  # noqa: E402

dev = torch.device("cuda", 0)
models = bench.build_models(dev, "bf16", 1234)
m, g, den, _, _ = models
for B in (6, 40):
    x, xl = bench.shard_inputs(0, 1, B, 1234 + B)
    torch.manual_seed(7)
    with torch.inference_mode():
        mel, yl, wav = bench.step(m, g, den, x.to(dev), xl.to(dev), 10, True)
    torch.cuda.synchronize()
    h = hashlib.sha256(mel.float().cpu().numpy().tobytes() + wav.float().cpu().numpy().tobytes()).hexdigest()[:16]
    print(f"syn_hash B={B}", h, float(wav.abs().max()))
