"""A/B of the decoder's hipGraph replay (mt_decoder_set_graphs) inside one process: synthesize() of the bench
shard (B=32, 10 Euler steps) alternating graphs on / off, median ms per call of each arm."""
import statistics
import sys
import time

import os as _os

_ROOT = _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))
sys.path.insert(0, _ROOT)
sys.path.insert(0, _os.path.join(_ROOT, "matcha-tts_amd"))

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    m, g, den, _, _ = bench.build_models(dev, "bf16", 1234)
    x, xl = bench.shard_inputs(0, 1, 32, 1234)
    x, xl = x.to(dev), xl.to(dev)
    eng = m.decoder.estimator.engine()
    res = {0: [], 1: []}
    for rep in range(12):
        for mode in (1, 0):
            eng.set_graphs(mode)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                m.synthesize(x, xl, n_timesteps=10, temperature=0.667)
            torch.cuda.synchronize()
            if rep >= 2:
                res[mode].append((time.perf_counter() - t0) / 3 * 1e3)
    eng.set_graphs(1)
    for mode in (1, 0):
        print(f"graphs={mode}: synthesize median {statistics.median(res[mode]):.3f} ms "
              f"(min {min(res[mode]):.3f})", flush=True)


if __name__ == "__main__":
    main()
