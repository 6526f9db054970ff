"""Time the CFM training step (matcha_hip.train.MatchaTrainer) at the reference's training shape: batch 64 per GPU
(train_standalone.py:760), LJSpeech-like lengths (mel frames ~ N(566, 150), text 150-250 tokens), synthetic
weights and data. Prints one JSON line: ms/step, mel frames/s, peak memory, and the per-phase split.

    python tools/train_bench.py [--batch 64] [--steps 5] [--warmup 2] [--no-dropout] [--precision 32|16-mixed|bf16-mixed]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "matcha-tts_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-dropout", action="store_true")
    ap.add_argument("--precision", default="32")
    a = ap.parse_args()
    from conftest import HP, make_matcha
    from matcha_hip import synthetic
    from matcha_hip.train import MatchaTrainer
    dev = torch.device("cuda")
    m = make_matcha(1, "fp32")
    sd = {k: torch.from_numpy(v) for k, v in synthetic.make_state_dict(
        [(k, tuple(v.shape)) for k, v in m.state_dict().items()], 1234).items()}
    B = a.batch
    yl = torch.as_tensor(synthetic.ljspeech_lengths(B, seed=1)).long()
    xl = (yl.float() / 3.0).clamp(20).long()  # ~3 frames per token
    Tx, Ty = int(xl.max()), int(-(-int(yl.max()) // 4) * 4)
    g = torch.Generator().manual_seed(0)
    x = torch.randint(1, 178, (B, Tx), generator=g) * (torch.arange(Tx)[None] < xl[:, None])
    y = torch.randn(B, 80, Ty, generator=g) * (torch.arange(Ty)[None, None] < yl[:, None, None])
    args = [t.to(dev) for t in (x, xl, y, yl)]
    tr = MatchaTrainer(sd, HP, dev, dropout=not a.no_dropout, precision=a.precision)
    for _ in range(a.warmup):
        tr.forward_backward(*args)
        tr.optimizer_step()
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        tr.forward_backward(*args)
        tr.optimizer_step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / a.steps
    frames = int(yl.sum())
    print(json.dumps({"what": "cfm_training_step", "batch": B, "Tx": Tx, "Ty": Ty, "mel_frames": frames,
                      "ms_per_step": round(ms, 2), "mel_frames_per_s": round(frames / ms * 1e3, 1),
                      "params": int(tr.params.flat.numel()), "peak_gb": round(torch.cuda.max_memory_allocated() / 1e9, 2),
                      "loss": round(float(tr.last["loss"]), 4), "dropout": not a.no_dropout,
                      "precision": a.precision, "loss_scale": tr.scaler["scale"] if tr.scaler else None}))


if __name__ == "__main__":
    main()
