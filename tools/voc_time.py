#!/usr/bin/env python3
"""Time the bench step's vocoder alone (bf16 Generator with the step's per-utterance lengths, i.e. the ragged
launch chain) on the mel the bench's synthesize produces. A/B knobs act through the environment (MT_LIB,
MT_XCD_TILES). Usage: python tools/voc_time.py [B] [reps]"""
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "matcha-tts_amd"))
sys.path.insert(0, HERE)

import torch  # noqa: E402

if os.environ.get("MT_LIB"):  # timing experiments: another build of the library
    import matcha_hip._lib as _L  # noqa: E402
    _L.LIB_PATH = os.environ["MT_LIB"]
import bench  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
dev = torch.device("cuda", 0)
m, g, den, _, _ = bench.build_models(dev, "bf16", 1234)
x, xl = bench.shard_inputs(0, 1, B, 1234)
x, xl = x.to(dev), xl.to(dev)
# VOC_CACHE=file.pt: the step's mel and lengths are read from it when it exists (written on the first run), so a
# library that lacks newer encoder / decoder entry points (MT_LIB, tools/ab_kern.sh) times the same vocoder input
cache = os.environ.get("VOC_CACHE")
with torch.inference_mode():
    if cache and os.path.exists(cache):
        d = torch.load(cache, weights_only=True)
        mel, yl = d["mel"].to(dev), d["yl"].to(dev)
    else:
        mel, yl, _ = m.synthesize(x, xl, n_timesteps=10, temperature=0.667, length_scale=1.0)
        if cache:
            torch.save({"mel": mel.cpu(), "yl": yl.cpu()}, cache)
    for _ in range(3):
        g(mel, lengths=yl)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g(mel, lengths=yl)
    e1.record()
    torch.cuda.synchronize()
print(f"vocoder ragged B={B} T={mel.shape[-1]}: {e0.elapsed_time(e1) / reps:.3f} ms")
