#!/usr/bin/env python3
"""Benchmark: text->wav mel-frames/s of the Matcha-TTS synthesis path on MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W`` prints ONE JSON line
on rank 0. For N>1 the driver launches one process per GPU with torch.distributed.run;
each rank synthesises its own shard of utterances (weak scaling, no data-path
collective: inference is embarrassingly parallel); a barrier +
synchronize brackets the timed region and the MAX over ranks is reported.

One step = the reference's text->wav call sequence on a batch (main.py:181-198 plus the
notebook denoiser, MOS_audiou_generator.ipynb:277): ``MatchaTTS.synthesize`` (HIP text encoder +
duration predictor in fp32, HIP duration/alignment path, HIP CFM 10-step Euler U-Net solver in bf16,
denormalize) -> ``Generator(mel).clamp(-1, 1)`` (HIP HiFi-GAN v1, bf16) -> ``Denoiser`` (HIP). The reference
vocodes and denoises one utterance per call on the mel `synthesize` cropped to it; the batched step does the same
for every utterance of the batch in one launch chain (``lengths=y_lengths``: each utterance at its own length,
identical to its one-utterance call, no columns past it computed).
Workload (configs[1] of BASELINE.json): 32 utterances/GPU, 10 ODE steps, bf16 MFMA;
synthetic LJSpeech-shaped text (x_len ~ U[150,251] with blanks) and synthetic weights
with the duration head forced to 3 frames/token -> 450..753 frames each.
``value`` = useful mel frames (sum of y_lengths) of all ranks / max-rank wall time.
Sub-records on rank 0 at N=1 (default workload): ``north_star`` (B=256 on one GPU), ``general_attention``
(a B=32 batch whose longest utterance is unpadded: the decoder's general attention path), ``batch1``
(batch-1 RTF as the reference's notebook times it), ``fp32_parity_mode`` and ``cpu_baseline``.
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


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--batch", type=int, default=32, help="utterances per GPU")
    p.add_argument("--n-timesteps", type=int, default=10)
    p.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    p.add_argument("--no-denoise", action="store_true")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-utterances", type=int, default=6, help="CPU baseline sample size (batch 1; ~20 s of CPU work)")
    p.add_argument("--no-north-star", action="store_true", help="skip the B=256 single-GPU record")
    p.add_argument("--no-fp32", action="store_true", help="skip the fp32 parity-mode record")
    p.add_argument("--quick", action="store_true", help="headline line only: no sub-record, no CPU baseline")
    p.add_argument("--seed", type=int, default=1234)
    p.add_argument("--model", default="lj", choices=["lj", "vctk"],
                   help="lj: single speaker (configs[1..2]); vctk: 109 speakers with the speaker-embedding "
                        "condition (configs[3]: B=128 over 8 GPUs = 16/GPU, 20 ODE steps)")
    # CPU rehearsal of the multi-rank launch (tests/test_bench_dist.py): gloo ranks, shards and the MAX / SUM
    # reduction with a host-side stand-in for the step; no GPU is touched
    p.add_argument("--cpu-selftest", action="store_true", help=argparse.SUPPRESS)
    return p.parse_args(argv)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv):
    """``--gpus N`` with no WORLD_SIZE in the environment: start N rank processes of this script, one per GPU, the
    way ``torch.distributed.run --nnodes 1 --nproc-per-node N --master-addr 127.0.0.1`` does (RANK, LOCAL_RANK,
    WORLD_SIZE, MASTER_ADDR / MASTER_PORT in each child's environment), and return the job's exit code (the first
    failing rank's; the other ranks are then stopped). The reference takes its device count from the CLI the same
    way (``devices=args.gpus``, train_standalone.py:763, 866-867). This parent never touches the GPU: it starts the
    children as fresh processes and only waits for them."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL on this driver
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    import signal

    def stop_all():  # every rank still alive: terminate, then kill after a grace period
        for q in procs:
            if q.poll() is None:
                q.terminate()
        deadline = time.time() + 10.0
        for q in procs:
            try:
                q.wait(timeout=max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                q.kill()

    def on_term(signum, frame):  # the driver's timeout: no orphaned ranks keep holding their GPUs
        stop_all()
        sys.exit(128 + signum)

    prev = signal.signal(signal.SIGTERM, on_term)
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for q in live:  # one rank failed: the job has failed, stop the ranks we started
                        q.terminate()
            time.sleep(0.05)
    finally:
        stop_all()
        signal.signal(signal.SIGTERM, prev)
    return rc


def build_models(device, precision, seed, n_spks=1):
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
    m = model.MatchaTTS(178, n_spks, 64, enc, dec, {"solver": "euler", "sigma_min": 1e-4}, dp, precision=precision)
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


def shard_speakers(rank, world, batch, seed, n_spks=109):
    """speaker ids of the shard's utterances (VCTK), drawn from the same global synthetic set"""
    ids = np.random.RandomState(seed + 17).randint(0, n_spks, size=batch * world)
    return torch.from_numpy(ids[rank * batch:(rank + 1) * batch].astype(np.int64))


def reduce_over_ranks(elapsed, frames, dist, device):
    """Job time = MAX of the ranks' timed regions; job work = SUM of their useful frames."""
    if dist is None:
        return elapsed, frames
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    f = torch.tensor([frames], dtype=torch.float64, device=device)
    dist.all_reduce(f, op=dist.ReduceOp.SUM)
    return float(t.item()), int(f.item())


def step(m, g, den, x, xl, n_ts, denoise, spk=None):
    spks = m.spk_emb(spk) if spk is not None else None  # main.py: the speaker embedding of the requested ids
    g.prepare(x.device)  # the vocoder's weight-cache check while the GPU runs synthesize, not after it
    mel, yl, attn = m.synthesize(x, xl, n_timesteps=n_ts, temperature=0.667, spks=spks, length_scale=1.0)
    # the reference's per-utterance vocoder + denoiser calls (main.py:198, MOS_audiou_generator.ipynb:276-277) for
    # the whole batch: utterance b at its own yl[b] frames
    wav = g(mel, lengths=yl).clamp(-1, 1)
    if denoise:
        wav = den(wav.squeeze(1), strength=0.00025, lengths=yl)
    return mel, yl, wav


# SURVEY.md §8d per-frame algorithmic cost of the hot path (one padded mel frame of one utterance):
# layer-boundary bytes (bf16) and FLOPs. Decoder per ODE step: 27,536 elements moved (25,488 GEMM-layer +
# 2,048 attention core) and 10,985,472 + 1,536*T + 6,619,136/T FLOPs; vocoder: 1,013,072 elements and
# 614,105,088 FLOPs per mel frame (exact).
DEC_BYTES_PER_FRAME_STEP = 27_536 * 2
VOC_BYTES_PER_FRAME = 1_013_072 * 2
VOC_FLOPS_PER_FRAME = 614_105_088
PEAK_FLOPS, PEAK_BW = 2.5e15, 8.0e12  # MI355X dense bf16 MFMA, HBM3E (MI355X_MICROARCH.md)


def dec_flops_per_frame_step(t_pad):
    return 10_985_472 + 1_536 * t_pad + 6_619_136 / t_pad


def path_roofline(sec_per_step, y_lengths, t_pad, n_ts):
    """Whole hot path (mu_y, mask, z -> wav): the roofline time of one step's work =
    max(FLOPs / MFMA peak, layer-boundary bytes / HBM peak), the decoder on B*T_pad frames x n_ts steps
    and the vocoder on its sum(y_lengths) frames (each utterance vocoded at its own length), over the measured
    step time. Also the verdict's useful-frames form:
    useful mel-frames/s over the bf16 HBM ceiling at T=576 (8e12 / 2,576,864 B = 3.10 M frames/s)."""
    B, t_y = len(y_lengths), max(y_lengths)
    dec_frames, voc_frames = B * t_pad, sum(y_lengths)
    flops = dec_frames * n_ts * dec_flops_per_frame_step(t_pad) + voc_frames * VOC_FLOPS_PER_FRAME
    nbytes = dec_frames * n_ts * DEC_BYTES_PER_FRAME_STEP + voc_frames * VOC_BYTES_PER_FRAME
    t_roof = max(flops / PEAK_FLOPS, nbytes / PEAK_BW)
    useful = sum(y_lengths) / sec_per_step
    ceiling = PEAK_BW / (10 * DEC_BYTES_PER_FRAME_STEP + VOC_BYTES_PER_FRAME)
    return {"bound": "hbm" if nbytes / PEAK_BW >= flops / PEAK_FLOPS else "mfma",
            "roof_ms_per_step": round(t_roof * 1e3, 3), "frac": round(t_roof / sec_per_step, 4),
            "tflops": round(flops / sec_per_step / 1e12, 1), "hbm_gbs": round(nbytes / sec_per_step / 1e9, 1),
            "decoder_frames_per_s": round(dec_frames / sec_per_step, 1),
            "useful_frames_per_s": round(useful, 1), "ceiling_frames_per_s_T576": round(ceiling, 1),
            "useful_frac_of_ceiling": round(useful / ceiling, 4), "padding_efficiency": round(sum(y_lengths) / dec_frames, 4),
            "scope": "hot path (decoder n_ts steps + vocoder); encoder and denoiser excluded as in SURVEY §8d"}


def _latest_profile(name):
    import glob
    files = sorted(glob.glob(os.path.join(HERE, "profiles", f"r*_{name}")))
    return files[-1] if files else None


def roofline_by_kernel(detail, frame_scale=1.0):
    """The family's launches split by kernel (mt_vconv: stage 1 and stage 2's k = 7 / 11 resblocks per layer;
    mt_vpair128: stage 2's k = 3 resblock as fused pairs; mt_vpair / mt_vpair32: stage 3 / 4
    pairs, priced as their two convs): mean launch ms, algorithmic rate on both sides and the fraction of the
    side the kernel's own intensity bounds it by."""
    out = {}
    for kind in ("rbconv", "vconv", "vpair128", "vpair", "vpair32", "rbfuse"):
        ls = [d for d in detail if d["kind"] == kind]
        if not ls:
            continue
        ms = sum(d["ms"] for d in ls)
        fl = sum(d["flops"] for d in ls) * frame_scale
        by = sum(d["bytes"] for d in ls) * frame_scale
        tf, gbs = fl / (ms * 1e-3) / 1e12, by / (ms * 1e-3) / 1e9
        mfma = fl / by >= PEAK_FLOPS / PEAK_BW
        out[kind] = {"launches": len(ls), "launch_ms": round(ms / len(ls), 4), "tflops": round(tf, 1),
                     "gbs": round(gbs, 1), "intensity_flop_per_byte": round(fl / by, 1),
                     "bound": "mfma" if mfma else "hbm",
                     "frac": round(tf / (PEAK_FLOPS / 1e12) if mfma else gbs / (PEAK_BW / 1e9), 4)}
    return out


def roofline(probe, default_workload=True, frame_scale=1.0, pmc_name="pmc_vconv.json"):
    """Dominant kernel family of the step: the LDS-DMA persistent implicit-GEMM convs that run every ResBlock
    conv of HiFi-GAN (51 launches per step): per layer on mt_rbconv (mt_vconv with MT_RBCONV=0), stage 1 and
    stage 2's k = 7 / 11 resblocks
    (30 convs; C = 256/128 on B x 8/64 * T_y frames); as fused conv pairs, stage 2's k = 3 resblock on
    mt_vpair128 (3 launches) and stages 3-4 on mt_vpair / mt_vpair32 (2 x 9 launches, C = 64/32 on
    B x 128/256 * T_y frames; a pair launch is priced as its two convs); k = 3/7/11. Timed by HIP events recorded on
    its launch stream around each of its launches in the LAST step of the timed region (mt_probe_*, site
    PROBE_VCONV). Per launch: algorithmic FLOPs = 2 * C_out * C_in * k * B * L;
    algorithmic bytes = layer-boundary bytes 2 * B * L * (C_in + C_out) (bf16 input read once, output
    written once) + weights. The family's intensity decides the bound against the bf16 ridge (2.5 PFLOP/s /
    8 TB/s = 312.5 FLOP/B). `roof_frac` = the summed per-launch roofline time max(F/P_mfma, B/P_hbm) over
    the measured time. The launches run ragged (each utterance at its own length): the host prices a launch on
    the padded B x L, so FLOPs, bytes and roof time are scaled by frame_scale = sum(y_lengths) / (B x T_y), the
    frames actually computed (the weight bytes, < 0.1 % of a launch's, scale with them).
    `traffic` = HBM bytes per launch from rocprofv3 FETCH_SIZE (x2, gfx950 correction)
    + WRITE_SIZE on this same bench command (profiles/rNN_pmc_vconv.json), `traffic_ratio` = traffic /
    algorithmic bytes (> 1: bytes this implementation moves beyond the layer boundaries)."""
    if probe is None or probe["launches"] == 0:
        return {"bound": "mfma", "achieved": None, "peak": 2500.0, "unit": "TFLOP/s", "frac": None,
                "traffic": None, "kernel": "vconv_kernel (bf16 path only)"}
    n = probe["launches"]
    ms = probe["ms"] / n
    flops = probe["flops"] / n * frame_scale
    nbytes = probe["bytes"] / n * frame_scale
    intensity = flops / nbytes
    tflops = flops / (ms * 1e-3) / 1e12
    gbs = nbytes / (ms * 1e-3) / 1e9
    peak_f, peak_b = PEAK_FLOPS / 1e12, PEAK_BW / 1e9
    ridge = PEAK_FLOPS / PEAK_BW
    traffic, pmc_file, stale = None, _latest_profile(pmc_name), None
    if pmc_file and default_workload:  # the PMC passes ran this workload (pmc_name: the default or the B=256 one)
        try:
            pmc = json.load(open(pmc_file))
            # only when they measured this run's family: same kernel sources and path knobs (tools/pmc_traffic.py)
            sys.path.insert(0, os.path.join(HERE, "tools"))
            from pmc_traffic import family_key
            if pmc.get("family_key") == family_key(HERE):
                traffic = pmc.get("hbm_bytes_per_launch")
            else:
                stale = f"{os.path.relpath(pmc_file, HERE)} measured another kernel build / path"
        except Exception:
            traffic = None
    if intensity >= ridge:
        bound, achieved, peak, unit = "mfma", tflops, peak_f, "TFLOP/s"
    else:
        bound, achieved, peak, unit = "hbm", gbs, peak_b, "GB/s"
    return {"bound": bound, "achieved": round(achieved, 2), "peak": peak, "unit": unit,
            "frac": round(achieved / peak, 4), "traffic": traffic,
            "traffic_ratio": round(traffic / nbytes, 3) if traffic else None,
            "traffic_source": os.path.relpath(pmc_file, HERE) if traffic else None,
            "traffic_stale": stale,
            "kernel": "LDS-DMA implicit-GEMM convs, HiFi-GAN stage 1-4 ResBlock convs: rbconv_kernel (stages 1-2 per layer, "
                      "compile-time K loop), vpair128 (stage 2 k=3 pairs), vpair / vpair32 (stages 3-4 pairs)",
            "launches": n, "launch_ms": round(ms, 4), "flops_per_launch": flops,
            "algo_bytes_per_launch": nbytes, "intensity_flop_per_byte": round(intensity, 1),
            "tflops": round(tflops, 2), "mfma_frac": round(tflops / peak_f, 4),
            "gbs": round(gbs, 1), "hbm_frac": round(gbs / peak_b, 4),
            "roof_frac": round(probe["roof_ms"] * frame_scale / probe["ms"], 4), "frame_scale": round(frame_scale, 4)}


def _cpu_info():
    model, phys = "unknown", set()
    try:
        cur = {}
        vis = os.sched_getaffinity(0)
        for line in open("/proc/cpuinfo"):
            if ":" not in line:
                if cur.get("processor") is not None and int(cur["processor"]) in vis:
                    phys.add((cur.get("physical id"), cur.get("core id")))
                cur = {}
                continue
            k, v = (s.strip() for s in line.split(":", 1))
            cur[k] = v
            if k == "model name":
                model = v
    except Exception:
        vis = set(range(os.cpu_count() or 1))
    return model, len(vis), len(phys) or len(vis)


def cpu_baseline(m_sd, g_sd, x, xl, n_ts, n_utt=3):
    """SURVEY.md §8d CPU baseline: the oracle (fp32 torch CPU restatement of the reference, "port") on a
    fixed sample of the same workload at batch 1, threads = the physical cores visible to this process
    (capped by OMP_NUM_THREADS, the box's CPU share), one warm-up pass, then the median of 3 timed passes.
    Two figures: BASELINE configs[0] exactly (B=1, 4 ODE steps, synthesise + Generator) and the bench's
    text->wav at n_ts steps with the denoiser."""
    from oracle import matcha_oracle as O
    from hifigan.config import v1
    model, visible, physical = _cpu_info()
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(physical, omp) if omp > 0 else physical
    torch.set_num_threads(threads)
    hp = dict(n_channels=192, n_layers=6, n_heads=2, kernel_size=3, dp_kernel_size=3, n_spks=1)
    sd = {k: v.detach().cpu() for k, v in m_sd.items()}
    gs = {k: v.detach().cpu() for k, v in g_sd.items()}
    bias = O.denoiser_bias_spec(gs, v1)
    g = torch.Generator().manual_seed(0)

    def run(steps, denoise):
        frames, t0 = 0, time.perf_counter()
        with torch.inference_mode():
            for n in range(n_utt):
                xi, li = x[n:n + 1, : int(xl[n])], xl[n:n + 1]
                mel, yl, _ = O.synthesize(sd, xi, li, steps, lambda mu: torch.randn(mu.shape, generator=g) * 0.667, hp)
                wav = O.generator_forward(gs, mel, v1).clamp(-1, 1)
                if denoise:
                    O.denoise(wav.squeeze(1), bias, 0.00025)
                frames += int(yl.sum())
        return frames, time.perf_counter() - t0

    out = {"unit": "mel-frames/s", "cores": threads, "kind": "port", "cpu_model": model,
           "visible_cpus": visible, "physical_cores_visible": physical}
    for key, steps, den in (("config1", 4, False), ("bench", n_ts, True)):
        run(steps, den)  # warm-up
        res = sorted((run(steps, den) for _ in range(3)), key=lambda r: r[1])
        frames, dt = res[1]
        out[key] = {"value": round(frames / dt, 2), "n_timesteps": steps, "denoiser": den,
                    "median_s": round(dt, 3), "runs_s": [round(r[1], 3) for r in res]}
    out["value"] = out["bench"]["value"]
    out["sample"] = (f"{n_utt} utterances of the bench shard at batch 1, fp32, {threads} threads; warm-up + median "
                     f"of 3. config1 = BASELINE configs[0] (B=1, 4 ODE steps, synthesise + Generator); bench = "
                     f"{n_ts} ODE steps text->wav + denoiser (the `value`)")
    return out


def north_star(m, g, den, batch, seed, n_ts, denoise, steps=10, warmup=2):
    """BASELINE north_star target point: B=256 utterances on ONE MI355X, 10-step text->wav, timed in this
    same run (its own warm-up; barrier-free single GPU)."""
    from matcha_hip import runtime as rt
    x_cpu, xl_cpu = shard_inputs(0, 1, batch, seed)
    x, xl = x_cpu.to(m.mel_mean.device), xl_cpu.to(m.mel_mean.device)
    for _ in range(warmup):
        step(m, g, den, x, xl, n_ts, denoise)
    _, yl, _ = step(m, g, den, x, xl, n_ts, denoise)
    yls = [int(v) for v in yl.cpu()]
    # the roofline family's launches of the LAST timed step are probed, as on the headline line
    rt.probe_start(rt.PROBE_VCONV, 64)
    rt.probe_pause(True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        if i == steps - 1:
            rt.probe_pause(False)
        step(m, g, den, x, xl, n_ts, denoise)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / steps
    detail = rt.probe_detail()
    probe = rt.probe_stop()
    t_pad = 4 * math.ceil(max(yls) / 4)
    fs = sum(yls) / (len(yls) * max(yls))
    roof = roofline(probe, default_workload=True, frame_scale=fs, pmc_name="pmc_vconv_b256.json")
    roof["by_kernel"] = roofline_by_kernel(detail, frame_scale=fs)
    return {"batch": batch, "steps": steps, "warmup": warmup, "ms_per_step": round(el * 1e3, 3),
            "value": round(sum(yls) / el, 2), "unit": "mel-frames/s", "seq_len": t_pad,
            "rtf": round(el / (sum(yls) * HOP / SR), 6), "roofline": roof,
            "path_roofline": path_roofline(el, yls, t_pad, n_ts)}


def timed_batch(m, g, den, x, xl, n_ts, denoise, steps, warmup):
    """mean seconds per step and the step's y_lengths, for one fixed batch already on the device"""
    for _ in range(warmup):
        step(m, g, den, x, xl, n_ts, denoise)
    _, yl, _ = step(m, g, den, x, xl, n_ts, denoise)
    yls = [int(v) for v in yl.cpu()]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step(m, g, den, x, xl, n_ts, denoise)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps, yls


def general_attention_record(m, g, den, batch, seed, n_ts, denoise, steps=10):
    """The bench batch with its longest texts clipped to a multiple of 4 tokens (3 frames per token -> the longest
    y_len % 4 == 0 -> T_pad = y_max, no padded frame in the longest utterance): the decoder's general Q.K^T
    attention path at both U-Net levels instead of the query-independent one (model.py:687-700, :1281). 4 of the
    8 shards of the 8-GPU configs[2] job are such batches (y_max 744, 744, 744, 732)."""
    x_cpu, xl_cpu = shard_inputs(0, 1, batch, seed)
    l4 = int(xl_cpu.max()) // 4 * 4
    xl_cpu = xl_cpu.clamp(max=l4)
    x_cpu = x_cpu[:, :l4].contiguous()
    dev = m.mel_mean.device
    el, yls = timed_batch(m, g, den, x_cpu.to(dev), xl_cpu.to(dev), n_ts, denoise, steps, 2)
    t_pad = 4 * math.ceil(max(yls) / 4)
    assert t_pad == max(yls)
    return {"batch": batch, "steps": steps, "ms_per_step": round(el * 1e3, 3), "value": round(sum(yls) / el, 2),
            "unit": "mel-frames/s", "seq_len": t_pad, "attention": "general (longest utterance unpadded)"}


def batch1_record(m, g, den, seed, n_ts, n_utt=10, reps=3):
    """The reference's only published number is batch-1 text->wav + denoiser RTF over 10 LJSpeech sentences
    (0.0173 on an unnamed CUDA GPU, MOS_audiou_generator.ipynb:257; upstream Matcha package and trained
    checkpoints, so context only): the same loop here, synchronising after every utterance as the notebook does."""
    x_all, xl_all = shard_inputs(0, 1, n_utt, seed + 99)
    dev = m.mel_mean.device
    rtf, lat, frames = [], [], 0
    for i in range(n_utt):
        x, xl = x_all[i:i + 1, : int(xl_all[i])].to(dev), xl_all[i:i + 1].to(dev)
        step(m, g, den, x, xl, n_ts, True)
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            _, yl, wav = step(m, g, den, x, xl, n_ts, True)
            wav.cpu()  # the notebook's .cpu() inside its timer
            ts.append(time.perf_counter() - t0)
        dt = sorted(ts)[len(ts) // 2]
        n = int(yl[0])
        frames += n
        lat.append(dt)
        rtf.append(dt / (n * HOP / SR))
    return {"utterances": n_utt, "n_timesteps": n_ts, "denoiser": True, "rtf_mean": round(sum(rtf) / n_utt, 6),
            "latency_ms_mean": round(1e3 * sum(lat) / n_utt, 3), "mel_frames_per_s": round(frames / sum(lat), 1),
            "published_rtf_context": 0.0173,
            "note": "median of 3 per utterance; published figure: unnamed CUDA GPU, upstream Matcha, trained weights"}


def fp32_record(device, seed, batch, n_ts, denoise, steps=3):
    """The parity mode (the reference's own fp32 arithmetic, exact-fp32 MFMA) on the bench workload."""
    m, g, den, _, _ = build_models(device, "fp32", seed)
    x_cpu, xl_cpu = shard_inputs(0, 1, batch, seed)
    el, yls = timed_batch(m, g, den, x_cpu.to(device), xl_cpu.to(device), n_ts, denoise, steps, 1)
    return {"batch": batch, "steps": steps, "ms_per_step": round(el * 1e3, 3), "value": round(sum(yls) / el, 2),
            "unit": "mel-frames/s", "dtype": "fp32",
            "ceiling_note": "fp32 MFMA 157.3 TF / 735 MFLOP per frame -> 214k frames/s (SURVEY.md §8d)"}


def cpu_selftest(a, world, rank):
    """--cpu-selftest: one rank of the launch contract on the CPU (gloo): the shard, a barrier-bracketed timed
    region around a host stand-in for the step, the MAX / SUM reduction and rank 0's JSON line"""
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    x, xl = shard_inputs(rank, world, a.batch, a.seed)
    frames = int(xl.sum()) * 3  # the forced duration head: 3 frames per token
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        torch.mm(torch.ones(64, 64), torch.ones(64, 64))
    if world > 1:
        dist.barrier()
    el, tot = reduce_over_ranks(time.perf_counter() - t0, frames, dist if world > 1 else None, torch.device("cpu"))
    if rank == 0:
        print(json.dumps({"metric": "cpu-selftest", "value": tot * a.steps / el, "n_gpus": world, "steps": a.steps,
                          "warmup": a.warmup, "frames_per_step": tot, "scaling": "weak"}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a.gpus, argv))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but the launcher started WORLD_SIZE={world} ranks", file=sys.stderr)
        sys.exit(2)
    if a.cpu_selftest:
        return cpu_selftest(a, world, rank)
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    torch.manual_seed(a.seed + rank)

    vctk = a.model == "vctk"
    from matcha_hip import _lib
    # a timing-experiment library (tools/exp_build.sh) computes wrong results; the loader refuses one already
    assert _lib.build_experiments() == 0, "bench.py needs a production build of libmatcha_hip.so"
    m, g, den, msd, gsd = build_models(device, a.precision, a.seed, n_spks=109 if vctk else 1)
    x_cpu, xl_cpu = shard_inputs(rank, world, a.batch, a.seed)
    x, xl = x_cpu.to(device), xl_cpu.to(device)
    spk = shard_speakers(rank, world, a.batch, a.seed).to(device) if vctk else None
    denoise = not a.no_denoise

    for _ in range(a.warmup):
        step(m, g, den, x, xl, a.n_timesteps, denoise, spk)
    torch.cuda.synchronize()

    # useful frames per step on this rank (deterministic durations), outside the timed region
    _, yl, wav = step(m, g, den, x, xl, a.n_timesteps, denoise, spk)
    yls = [int(v) for v in yl.cpu()]
    frames = int(yl.sum())
    t_y = int(yl.max())
    t_pad = 4 * math.ceil(t_y / 4)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    from matcha_hip import runtime as rt
    # the probe brackets the family's launches of the LAST timed step only: each event pair leaves a few
    # microseconds of idle before its launch, so the other timed steps run unprobed
    rt.probe_start(rt.PROBE_VCONV, 64)
    rt.probe_pause(True)
    barrier()
    t0 = time.perf_counter()
    for i in range(a.steps):
        if i == a.steps - 1:
            rt.probe_pause(False)
        step(m, g, den, x, xl, a.n_timesteps, denoise, spk)
    barrier()
    el = time.perf_counter() - t0
    detail = rt.probe_detail()
    probe = rt.probe_stop()

    el, tot_frames = reduce_over_ranks(el, frames, dist, device)

    value = tot_frames * a.steps / el
    ms_per_step = el / a.steps * 1e3
    audio_s = tot_frames * HOP / SR
    out = {
        "metric": "mel-frames/sec + RTF, text->wav @10 ODE steps, LJSpeech model, 1/2/4/8 GPU" if not vctk else
                  f"mel-frames/sec + RTF, text->wav @{a.n_timesteps} ODE steps, VCTK 109-speaker model",
        "value": round(value, 2), "unit": "mel-frames/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": a.precision,
        "data": "synthetic (random-init weights, LJSpeech-shaped text; duration head forced to 3 frames/token)",
        "config": {"workload": f"text->wav: synthesize({a.n_timesteps}-step Euler CFM) + HiFi-GAN v1 + denoiser"
                               + (" (VCTK, speaker-embedding condition)" if vctk else ""),
                   "global_batch": a.batch * world, "batch_per_gpu": a.batch, "n_timesteps": a.n_timesteps,
                   "seq_len": t_pad, "frames_per_step": tot_frames, "parallelism": f"dp{world} (utterance shards)",
                   "denoiser": denoise, "vocoder": "each utterance at its own length (ragged batch, = its one-utterance call)"},
        "rtf": round((el / a.steps) / audio_s, 6),
        "build_experiments": _lib.build_experiments(),
    }
    if rank == 0:
        if world == 1:
            default = (a.batch, a.n_timesteps, a.seed, a.no_denoise, a.precision, a.model) == \
                (32, 10, 1234, False, "bf16", "lj")
            fs = sum(yls) / (len(yls) * max(yls))  # ragged vocoder: frames computed / padded frames priced
            out["roofline"] = roofline(probe, default_workload=default, frame_scale=fs)
            out["roofline"]["by_kernel"] = roofline_by_kernel(detail, frame_scale=fs)
            out["path_roofline"] = path_roofline(el / a.steps, yls, t_pad, a.n_timesteps)
            if a.quick:
                a.no_north_star = a.no_cpu_baseline = a.no_fp32 = True
            if default and not a.quick:
                out["general_attention"] = general_attention_record(m, g, den, a.batch, a.seed, a.n_timesteps,
                                                                    denoise)
                out["batch1"] = batch1_record(m, g, den, a.seed, a.n_timesteps)
            if not a.no_north_star and a.batch != 256 and a.precision == "bf16" and not vctk:
                out["north_star"] = north_star(m, g, den, 256, a.seed, a.n_timesteps, denoise)
            if default and not a.no_fp32:
                out["fp32_parity_mode"] = fp32_record(device, a.seed, a.batch, a.n_timesteps, denoise)
            if not a.no_cpu_baseline and not vctk:
                out["cpu_baseline"] = cpu_baseline(msd, gsd, x_cpu, xl_cpu, a.n_timesteps, a.cpu_utterances)
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
