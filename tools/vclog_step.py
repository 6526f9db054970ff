#!/usr/bin/env python3
"""Every mt_vconv launch of one bench step (B from argv, default 32), grouped by variant: epilogue flags, tile rows /
frames, 1x1 mode, taps, C_out, C_in, tile count, grid, launches. Usage: python tools/vclog_step.py [B]"""
import os
import sys
from collections import Counter

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "matcha-tts_amd"))
sys.path.insert(0, HERE)
import torch  # noqa: E402

import bench  # noqa: E402
from matcha_hip import runtime as rt  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
dev = torch.device("cuda", 0)
m, g, den, _, _ = bench.build_models(dev, "bf16", 1234)
x, xl = bench.shard_inputs(0, 1, B, 1234)
x, xl = x.to(dev), xl.to(dev)
with torch.inference_mode():
    bench.step(m, g, den, x, xl, 10, True)
    torch.cuda.synchronize()
    rt.vconv_log_start(100000)
    bench.step(m, g, den, x, xl, 10, True)
    torch.cuda.synchronize()
    recs = rt.vconv_log_stop(100000)
cnt = Counter()
for r in recs:
    ef, bm, bn, k1, ntiles, grid, taps, M, cin, b, L = (r[f] for f in rt.VCONV_LOG_FIELDS)
    cnt[(ef, bm, bn, k1, taps, M, cin, ntiles, grid)] += 1
print("ef bm bn k1 taps M cin ntiles grid : launches")
for k, v in sorted(cnt.items(), key=lambda kv: -kv[1]):
    print(*k, ":", v)
