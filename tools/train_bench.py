"""Time the CFM training step (matcha_hip.train.MatchaTrainer) at the reference's training shape: batch 64 per GPU
(train_standalone.py:760), LJSpeech-like lengths (mel frames ~ N(566, 150), text 150-250 tokens), synthetic
weights and data. Prints one JSON line: ms/step, mel frames/s, peak memory, and the step's MFMA roofline (FLOPs of
its GEMMs / convs / attention against the precision's MFMA peak).

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


def step_flops(B, Tx, Ty):
    """GEMM / conv / attention FLOPs of one training step (forward x 3: forward, data and weight gradients) on the
    padded shapes the step computes: the text encoder + duration predictor on B x Tx tokens (prenet 3 x k = 5 convs +
    1x1, 6 RoPE layers: QKV, attention 2 x 2 x Tx x 192 per token, out-projection, FFN k = 3 192 <-> 768; proj_m;
    duration predictor k = 3 192 -> 256 -> 256 -> 1), and one estimator evaluation on B x Ty frames (bench.py's
    per-frame decoder count)."""
    import bench
    c, f, dp = 192, 768, 256
    enc = (3 * 2 * c * c * 5 + 2 * c * c
           + 6 * (3 * 2 * c * c + 2 * c * c + 2 * 2 * Tx * c + 2 * (2 * c * f * 3))
           + 2 * c * 80 + 2 * c * dp * 3 + 2 * dp * dp * 3 + 2 * dp)
    return 3 * (B * Tx * enc + B * Ty * bench.dec_flops_per_frame_step(Ty))


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
    sys.path.insert(0, ROOT)
    flops = step_flops(B, Tx, Ty)
    # the GEMM operands' arithmetic: exact fp32 MFMA (157.3 TF) in "32", fp16 / bf16 MFMA (2.5 PF dense) when mixed
    peak = 157.3e12 if a.precision == "32" else 2.5e15
    print(json.dumps({"what": "cfm_training_step", "batch": B, "Tx": Tx, "Ty": Ty, "mel_frames": frames,
                      "ms_per_step": round(ms, 2), "mel_frames_per_s": round(frames / ms * 1e3, 1),
                      "params": int(tr.params.flat.numel()), "peak_gb": round(torch.cuda.max_memory_allocated() / 1e9, 2),
                      "loss": round(float(tr.last["loss"]), 4), "dropout": not a.no_dropout,
                      "precision": a.precision, "loss_scale": tr.scaler["scale"] if tr.scaler else None,
                      "roofline": {"bound": "mfma", "gflop_per_step": round(flops / 1e9, 1),
                                   "achieved_tflops": round(flops / ms / 1e9, 1), "peak_tflops": peak / 1e12,
                                   "frac": round(flops / ms / 1e9 / (peak / 1e12), 4),
                                   "scope": "GEMM / conv / attention FLOPs x 3 on the padded shapes; the elementwise, "
                                            "normalisation, MAS and optimizer work is not priced"}}))


if __name__ == "__main__":
    main()
