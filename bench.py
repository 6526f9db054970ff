#!/usr/bin/env python3
"""Benchmark: text->wav mel-frames/s of the Matcha-TTS synthesis path on MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W`` prints ONE JSON line
on rank 0. For N>1 the driver launches one process per GPU with torch.distributed.run;
each rank synthesises its own shard of utterances (weak scaling, no data-path
collective: inference is embarrassingly parallel); a barrier +
synchronize brackets the timed region and the MAX over ranks is reported.

One step = the reference's text->wav call sequence on a batch (main.py:181-198 plus the
notebook denoiser, MOS_audiou_generator.ipynb:277): ``MatchaTTS.synthesize`` (host-PyTorch
text encoder, HIP duration/alignment path, HIP CFM 10-step Euler U-Net solver,
denormalize) -> ``Generator(mel).clamp(-1, 1)`` (HIP HiFi-GAN v1) -> ``Denoiser`` (HIP).
Workload (configs[1] of BASELINE.json): 32 utterances/GPU, 10 ODE steps, bf16 MFMA;
synthetic LJSpeech-shaped text (x_len ~ U[150,251] with blanks) and synthetic weights
with the duration head forced to 3 frames/token -> 450..753 frames each.
``value`` = useful mel frames (sum of y_lengths) of all ranks / max-rank wall time.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "matcha-tts_amd"))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402

SR, HOP = 22050, 256


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--batch", type=int, default=32, help="utterances per GPU")
    p.add_argument("--n-timesteps", type=int, default=10)
    p.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    p.add_argument("--no-denoise", action="store_true")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=15.0)
    p.add_argument("--seed", type=int, default=1234)
    return p.parse_args()


def build_models(device, precision, seed):
    from types import SimpleNamespace

    import model
    from hifigan.config import v1
    from hifigan.denoiser import Denoiser
    from hifigan.env import AttrDict
    from hifigan.models import Generator
    from matcha_hip import synthetic

    enc = SimpleNamespace(encoder_type="RoPE Encoder", n_feats=80, n_channels=192, filter_channels=768, n_heads=2,
                          n_layers=6, kernel_size=3, p_dropout=0.1, prenet=True)
    dec = SimpleNamespace(channels=(256, 256), dropout=0.05, attention_head_dim=64, n_blocks=1, num_mid_blocks=2,
                          num_heads=2, act_fn="snakebeta")
    dp = SimpleNamespace(filter_channels_dp=256, kernel_size=3, p_dropout=0.1)
    m = model.MatchaTTS(178, 1, 64, enc, dec, {"solver": "euler", "sigma_min": 1e-4}, dp, precision=precision)
    sd = synthetic.make_state_dict([(k, tuple(v.shape)) for k, v in m.state_dict().items()], seed,
                                   force_log_duration=math.log(2.5))
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m = m.to(device).eval()
    g = Generator(AttrDict(v1), precision=precision)
    gsd = synthetic.make_state_dict([(k, tuple(v.shape)) for k, v in g.state_dict().items()], seed + 7)
    g.load_state_dict({k: torch.from_numpy(v) for k, v in gsd.items()})
    g = g.to(device).eval()
    g.remove_weight_norm()
    den = Denoiser(g, mode="zeros")
    return m, g, den, {k: torch.from_numpy(v) for k, v in sd.items()}, dict(g.state_dict())


def shard_inputs(rank, world, batch, seed):
    """Rank r gets utterances [r*batch, (r+1)*batch) of one global synthetic set of world*batch
    utterances (weak scaling: the per-GPU batch is fixed), cropped to the shard's longest text."""
    from matcha_hip import synthetic
    x, xl = synthetic.synthetic_text(batch * world, seed=seed)
    x, xl = x[rank * batch:(rank + 1) * batch], xl[rank * batch:(rank + 1) * batch]
    x = x[:, : int(xl.max())]
    return torch.from_numpy(np.ascontiguousarray(x)), torch.from_numpy(np.ascontiguousarray(xl))


def reduce_over_ranks(elapsed, frames, dist, device):
    """Job time = MAX of the ranks' timed regions; job work = SUM of their useful frames."""
    if dist is None:
        return elapsed, frames
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    f = torch.tensor([frames], dtype=torch.float64, device=device)
    dist.all_reduce(f, op=dist.ReduceOp.SUM)
    return float(t.item()), int(f.item())


def step(m, g, den, x, xl, n_ts, denoise):
    mel, yl, attn = m.synthesize(x, xl, n_timesteps=n_ts, temperature=0.667, length_scale=1.0)
    wav = g(mel).clamp(-1, 1)
    if denoise:
        wav = den(wav.squeeze(1), strength=0.00025)
    return mel, yl, wav


def roofline(probe, precision, default_workload=True):
    """Dominant kernel of the step: mt_vconv, the LDS-DMA persistent implicit-GEMM conv that runs every
    ResBlock conv of HiFi-GAN stages 1-3 (54 launches per step: 3 stages x 3 resblocks x 3 pairs x
    2 convs; C = 256/128/64 on B x 8/64/128 * T_y frames, k = 3/7/11). Timed by HIP events recorded on
    its launch stream around each of its launches INSIDE the timed region (mt_probe_*, site
    PROBE_VCONV). Per launch: algorithmic FLOPs = 2 * C_out * C_in * k * B * L; algorithmic bytes =
    input + output (+ residual, + accumulator, + activated copy) activations of B * L frames x C
    channels in bf16, + weights (mt_vconv.hip launch_vconv). The family's intensity decides the bound:
    below the bf16 ridge (2.5 PFLOP/s / 8 TB/s = 312.5 FLOP/B) it is HBM-bound and `achieved` is
    algorithmic GB/s, above it MFMA-bound and `achieved` is TFLOP/s. `traffic` = HBM bytes per launch
    from rocprofv3 FETCH_SIZE (x2, gfx950 correction) + WRITE_SIZE on this same bench command
    (profiles/r01_pmc_vconv.json, tools_round_profile.sh)."""
    if probe is None or probe["launches"] == 0:
        return {"bound": "hbm", "achieved": None, "peak": 8000.0, "unit": "GB/s", "frac": None,
                "traffic": None, "kernel": "vconv_kernel (bf16 path only)"}
    n = probe["launches"]
    ms = probe["ms"] / n
    flops = probe["flops"] / n
    nbytes = probe["bytes"] / n
    intensity = flops / nbytes
    tflops = flops / (ms * 1e-3) / 1e12
    gbs = nbytes / (ms * 1e-3) / 1e9
    peak_f, peak_b = 2500.0, 8000.0  # dense bf16 MFMA TFLOP/s, HBM GB/s (MI355X_MICROARCH.md)
    ridge = peak_f * 1e12 / (peak_b * 1e9)
    traffic = None
    pmc = os.path.join(HERE, "profiles", "r01_pmc_vconv.json")
    if os.path.exists(pmc) and default_workload:  # the PMC passes ran the default bench workload only
        try:
            traffic = json.load(open(pmc)).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    if intensity >= ridge:
        bound, achieved, peak, unit = "mfma", tflops, peak_f, "TFLOP/s"
    else:
        bound, achieved, peak, unit = "hbm", gbs, peak_b, "GB/s"
    return {"bound": bound, "achieved": round(achieved, 2), "peak": peak, "unit": unit,
            "frac": round(achieved / peak, 4), "traffic": traffic,
            "kernel": "vconv_kernel<bf16> LDS-DMA implicit-GEMM conv, HiFi-GAN stage 1-3 ResBlock convs",
            "launches": n, "launch_ms": round(ms, 4), "flops_per_launch": flops,
            "algo_bytes_per_launch": nbytes, "intensity_flop_per_byte": round(intensity, 1),
            "tflops": round(tflops, 2), "mfma_frac": round(tflops / peak_f, 4),
            "gbs": round(gbs, 1), "hbm_frac": round(gbs / peak_b, 4)}


def cpu_baseline(m_sd, g_sd, x, xl, n_ts, seconds):
    """Oracle (torch CPU restatement, fp32) on a bounded sample of the same workload."""
    from oracle import matcha_oracle as O
    from hifigan.config import v1
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    hp = dict(n_channels=192, n_layers=6, n_heads=2, kernel_size=3, dp_kernel_size=3, n_spks=1)
    sd = {k: v.detach().cpu() for k, v in m_sd.items()}
    gs = {k: v.detach().cpu() for k, v in g_sd.items()}
    bias = O.denoiser_bias_spec(gs, v1)
    frames, n, t0 = 0, 0, time.perf_counter()
    with torch.inference_mode():
        while n < x.shape[0]:
            xi, li = x[n:n + 1, : int(xl[n])], xl[n:n + 1]
            mel, yl, _ = O.synthesize(sd, xi, li, n_ts, lambda mu: torch.randn_like(mu) * 0.667, hp)
            wav = O.generator_forward(gs, mel, v1).clamp(-1, 1)
            O.denoise(wav.squeeze(1), bias, 0.00025)
            frames += int(yl.sum())
            n += 1
            if time.perf_counter() - t0 > seconds:
                break
    dt = time.perf_counter() - t0
    return {"value": round(frames / dt, 2), "unit": "mel-frames/s", "cores": threads, "kind": "port",
            "sample": f"{n} utterance(s) x {n_ts} ODE steps text->wav (+denoiser), batch 1, fp32, "
                      f"{frames} frames in {dt:.1f}s"}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    torch.manual_seed(a.seed + rank)

    m, g, den, msd, gsd = build_models(device, a.precision, a.seed)
    x_cpu, xl_cpu = shard_inputs(rank, world, a.batch, a.seed)
    x, xl = x_cpu.to(device), xl_cpu.to(device)
    denoise = not a.no_denoise

    for _ in range(a.warmup):
        step(m, g, den, x, xl, a.n_timesteps, denoise)
    torch.cuda.synchronize()

    # useful frames per step on this rank (deterministic durations), outside the timed region
    _, yl, wav = step(m, g, den, x, xl, a.n_timesteps, denoise)
    frames = int(yl.sum())
    t_y = int(yl.max())
    t_pad = 4 * math.ceil(t_y / 4)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    from matcha_hip import runtime as rt
    rt.probe_start(rt.PROBE_VCONV, 64 * a.steps)
    barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(m, g, den, x, xl, a.n_timesteps, denoise)
    barrier()
    el = time.perf_counter() - t0
    probe = rt.probe_stop()

    el, tot_frames = reduce_over_ranks(el, frames, dist, device)

    value = tot_frames * a.steps / el
    ms_per_step = el / a.steps * 1e3
    audio_s = tot_frames * HOP / SR
    out = {
        "metric": "mel-frames/sec + RTF, text->wav @10 ODE steps, LJSpeech model, 1/2/4/8 GPU",
        "value": round(value, 2), "unit": "mel-frames/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": a.precision,
        "data": "synthetic (random-init weights, LJSpeech-shaped text; duration head forced to 3 frames/token)",
        "config": {"workload": "text->wav: synthesize(10-step Euler CFM) + HiFi-GAN v1 + denoiser",
                   "global_batch": a.batch * world, "batch_per_gpu": a.batch, "n_timesteps": a.n_timesteps,
                   "seq_len": t_pad, "frames_per_step": tot_frames, "parallelism": f"dp{world} (utterance shards)",
                   "denoiser": denoise},
        "rtf": round((el / a.steps) / audio_s, 6),
    }
    if rank == 0:
        if world == 1:
            default = (a.batch, a.n_timesteps, a.seed, a.no_denoise, a.precision) == (32, 10, 1234, False, "bf16")
            out["roofline"] = roofline(probe, a.precision, default_workload=default)
            if not a.no_cpu_baseline:
                out["cpu_baseline"] = cpu_baseline(msd, gsd, x_cpu, xl_cpu, a.n_timesteps, a.cpu_seconds)
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
