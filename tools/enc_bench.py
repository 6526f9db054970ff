#!/usr/bin/env python3
"""Time the text encoder + duration predictor alone on the bench's text batch (fp32 by default, as the bf16 model
runs it). Usage: python tools/enc_bench.py [B] [reps] [precision]"""
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
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
prec = sys.argv[3] if len(sys.argv) > 3 else "fp32"
dev = torch.device("cuda", 0)
m, _, _, _, _ = bench.build_models(dev, "bf16", 1234)
m.set_precision("bf16", encoder_precision=prec)
x, xl = bench.shard_inputs(0, 1, B, 1234)
x, xl = x.to(dev), xl.to(dev)
with torch.inference_mode():
    for _ in range(3):
        m.encoder(x, xl)  # checked once (OOV ids raise), then timed without the per-call host sync
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        m.encoder.forward_unchecked(x, xl)
    e1.record()
    torch.cuda.synchronize()
print(f"encoder {prec} B={B} Tx={x.shape[1]}: {e0.elapsed_time(e1) / reps:.3f} ms")
