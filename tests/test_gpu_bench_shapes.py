"""Parity at the shapes the bench times (MI355X).

The headline number comes from kernel variants that tiny test shapes never select: mt_vconv picks
its tile width / pipeline from the problem size and runs a persistent grid of one workgroup per CU,
so only grids with more tiles than CUs exercise the multi-tile walk (cross-tile prefetch, the
``nmine >= 2`` loop, the XCD remap). These tests run

  (a) one bf16 estimator evaluation at the bench shape (B=32, T=728) and at B=128 (every k=3
      GroupNorm conv multi-tile), whole batch against the fp32 oracle;
  (b) the bf16 Generator at B=8, T=728 (stage-1 convs with 368 tiles, stages 2-3 >1000 tiles);
  (c) the exact bench step (bf16 text->wav: encoder, 10-step Euler CFM, HiFi-GAN, denoiser) at
      B=32 and at the north-star batch B=256, rows against the oracle run on those rows at the
      batch's padded length (rows are independent given T_pad and their z slice), the
      vocoder and denoiser per utterance on its cropped mel as the reference calls them (the step's ragged
      vocoder: tests/test_gpu_ragged.py);
  (d) an fp32 10-step CFM solve against the oracle,

and record every mt_vconv launch (variant + grid) so the last test can assert that each variant
the bench step launches was parity-checked here with a multi-tile grid whenever the bench runs it
multi-tile. Tolerances: bf16 vs the fp32 oracle by relative RMS 1e-2 (the SURVEY §8c bf16 bar) on the
estimator, generator waveform and on the bench rows' mel and denoised waveform (measured on MI355X: 9.7e-3,
5.5e-3, 5.7e-3 and 9.6e-3; the reference's own autocast-bf16 on the same weights: 1.1e-2 for one estimator
evaluation, 6.6e-3 on the Generator — tests/test_gpu_parity_bf16.py); the text encoder runs fp32 in the bf16
model (mu 1e-4); fp32 CFM atol 2e-4 (SURVEY §8c fp32 mode; measured 3.9e-6).
Reference: model.py:964-1048, 1084-1109, 1264-1300; hifigan/models.py:181-197;
hifigan/denoiser.py:62-68.
"""
import math
import os
import sys

import numpy as np
import pytest
import torch

from conftest import REPO, make_decoder, make_generator, rel_rms

pytestmark = pytest.mark.gpu
DEV = "cuda"
LOGS = {}  # test name -> vconv launch records


def _variant(r):
    return (r["ef"], r["bm"], r["bn"], r["k1"], r["taps"])


def _synth_sd(mod, seed):
    from matcha_hip import synthetic
    return {k: torch.from_numpy(v) for k, v in synthetic.make_state_dict(
        [(k, tuple(v.shape)) for k, v in mod.state_dict().items()], seed).items()}


def _bench():
    if REPO not in sys.path:
        sys.path.insert(0, REPO)
    import bench
    return bench


# ------------------------------------------------------------------------------- (a) estimator
@pytest.mark.parametrize("B", [32, 128])
def test_decoder_bf16_step_bench_shape_vs_oracle(B):
    from matcha_hip import runtime as rt
    from oracle import matcha_oracle as O
    dec = make_decoder(160, "bf16")
    sd = _synth_sd(dec, 5)
    dec.load_state_dict(sd)
    dec = dec.to(DEV).eval()
    T = 728
    rs = np.random.RandomState(B)
    lens = np.clip(np.round(rs.normal(566, 150, B)), 96, T).astype(np.int64)
    lens[0] = T  # one unpadded row (the mask quirk inactive there), the rest ragged
    g = torch.Generator().manual_seed(B)
    x, mu = torch.randn(B, 80, T, generator=g) * 0.667, torch.randn(B, 80, T, generator=g)
    mask = (torch.arange(T)[None] < torch.from_numpy(lens)[:, None]).float()[:, None]
    tt = torch.full((B,), 0.3)
    rt.vconv_log_start()
    out = dec(x.to(DEV), mask.to(DEV), (mu * mask).to(DEV), tt.to(DEV)).cpu()
    torch.cuda.synchronize()
    LOGS[f"decoder{B}"] = rt.vconv_log_stop()
    ref = O.decoder_forward(sd, x, mask, mu * mask, tt)
    err = rel_rms(out, ref)
    rows = [rel_rms(out[i], ref[i]) for i in range(B)]
    worst = max(rows)
    # the reference's own bf16 mode (torch.autocast over the same ops) on the same inputs, row by row
    with torch.inference_mode(), torch.autocast("cpu", dtype=torch.bfloat16):
        ac = O.decoder_forward(sd, x, mask, mu * mask, tt).float()
    ac_rows = [rel_rms(ac[i], ref[i]) for i in range(B)]
    print(f"decoder B={B} T={T}: rel-RMS {err:.3e}, worst row {worst:.3e}; reference autocast-bf16 {rel_rms(ac, ref):.3e}, "
          f"worst row {max(ac_rows):.3e}; rows worse than autocast: {sum(a > b for a, b in zip(rows, ac_rows))}/{B}")
    assert torch.isfinite(out).all()
    # the whole batch within the §8c bar; every row no worse than the reference's own bf16 mode on that row (a
    # short, mostly padded row reaches ~1e-2 in both: measured worst 1.02e-2 here vs 1.14e-2 under autocast)
    assert err < 1e-2, err
    assert all(r <= a for r, a in zip(rows, ac_rows)), [(i, r, a) for i, (r, a) in enumerate(zip(rows, ac_rows)) if r > a]
    gn = [r for r in LOGS[f"decoder{B}"] if r["ef"] & 256]
    # tile widths by the cost model: B=32 -> 192 (full resolution, exactly 256 tiles) and 128 (half);
    # B=128 -> 256 (full) and 192 (half), both multi-tile as at the north-star batch
    want = {32: {128, 192}, 128: {192, 256}}[B]
    assert {r["bn"] for r in gn} == want, ({r["bn"] for r in gn}, want)
    if B == 128:
        assert all(r["ntiles"] > r["grid"] for r in gn), "GroupNorm convs must walk several tiles"


@pytest.mark.parametrize("enc_precision", ["fp32", "bf16"])
@pytest.mark.parametrize("B", [32, 256])
def test_text_encoder_bench_batch_vs_oracle(B, enc_precision):
    """The bench's text batch (x_len ~ U[150,251] with blanks) through the text encoder. fp32 is what the bf16
    model runs (model.MatchaTTS: the index path needs the reference's fp32 logw): mu within 1e-4. bf16 is the
    opt-in ``encoder_precision="bf16"`` mode, off the product path: its FFN convs run on mt_vconv (multi-tile at
    B=256) and its bar is the 2e-2 this mode was built to (mu measured 1.1e-2), not the §8c contract."""
    from matcha_hip import runtime as rt
    from oracle import matcha_oracle as O
    bench = _bench()
    m, _, _, msd, _ = bench.build_models(torch.device(DEV), "bf16", 1234)
    m.set_precision("bf16", encoder_precision=enc_precision)
    x, xl = bench.shard_inputs(0, 1, B, 1234)
    rt.vconv_log_start()
    mu, logw, xm = m.encoder(x.to(DEV), xl.to(DEV))
    torch.cuda.synchronize()
    LOGS[f"encoder{B}_{enc_precision}"] = rt.vconv_log_stop()
    sd = {k[len("encoder."):]: v.cpu() for k, v in msd.items() if k.startswith("encoder.")}
    mu_o, logw_o, xm_o = O.text_encoder(sd, x, xl, dict(n_channels=192, n_layers=6, n_heads=2, kernel_size=3,
                                                        dp_kernel_size=3, n_spks=1))
    assert torch.equal(xm.cpu(), xm_o) and torch.equal(logw.cpu(), logw_o)
    err = rel_rms(mu.cpu(), mu_o)
    print(f"encoder {enc_precision} B={B} Tx={x.shape[1]}: mu rel-RMS {err:.3e}")
    assert err < (1e-4 if enc_precision == "fp32" else 2e-2), err


# ------------------------------------------------------------------------------- (b) generator
def test_generator_bf16_bench_length_vs_oracle():
    from hifigan.config import v1
    from matcha_hip import runtime as rt
    from oracle import matcha_oracle as O
    gen = make_generator("bf16")
    gen.load_state_dict(_synth_sd(gen, 8))
    gen = gen.to(DEV).eval()
    gen.remove_weight_norm()
    B, T = 8, 728
    mel = torch.randn(B, 80, T, generator=torch.Generator().manual_seed(9)) * 2.1 - 5.5
    rt.vconv_log_start()
    wav = gen(mel.to(DEV)).cpu()
    torch.cuda.synchronize()
    LOGS["generator"] = rt.vconv_log_stop()
    ref = O.generator_forward({k: v.cpu() for k, v in gen.state_dict().items()}, mel, v1)
    err = rel_rms(wav, ref)
    worst = max(rel_rms(wav[i], ref[i]) for i in range(B))
    print(f"generator B={B} T={T}: rel-RMS {err:.3e}, worst row {worst:.3e}")
    assert err < 1e-2 and worst < 1e-2, (err, worst)
    # stage 1 + stage 2's k = 7 / 11 resblocks: 30 per-layer ResBlock convs; stage 2's k = 3 resblock: 3 fused pairs
    # (mt_vpair128); stages 3-4: 9 fused pairs each (mt_vpair / mt_vpair32); fused launches log ef | 0x10000
    res = [r for r in LOGS["generator"] if not r["k1"] and r["taps"] >= 3]
    assert len(res) == 30 + 21 and sum(1 for r in res if r["ef"] & 0x10000) == 21
    assert all(r["ntiles"] > r["grid"] for r in res), \
        [(r["M"], r["ntiles"], r["grid"]) for r in res if r["ntiles"] <= r["grid"]]


# ------------------------------------------------------------------------------- (c) bench step
def _bench_rows_vs_oracle(batch, rows, tag, rank=0, world=1, vctk=False, n_ts=10, inputs=None, row_bar=1e-2,
                          solver="euler"):
    from hifigan.config import v1
    from matcha_hip import runtime as rt
    from oracle import matcha_oracle as O
    bench = _bench()
    n_spks = 109 if vctk else 1
    m, g, den, msd, gsd = bench.build_models(torch.device(DEV), "bf16", 1234, n_spks=n_spks)
    m.decoder.solver = solver
    x, xl = bench.shard_inputs(rank, world, batch, 1234) if inputs is None else inputs
    spk = bench.shard_speakers(rank, world, batch, 1234).to(DEV) if vctk else None
    torch.manual_seed(1234 + rank)  # bench.main's per-rank noise seed
    real = torch.randn_like
    zs = []

    def noise(ref, *a, **k):
        zs.append(real(ref))
        return zs[-1].clone()

    torch.randn_like = noise
    try:
        rt.vconv_log_start()
        mel, yl, wav = bench.step(m, g, den, x.to(DEV), xl.to(DEV), n_ts, True, spk)
        torch.cuda.synchronize()
        LOGS[tag] = rt.vconv_log_stop()
    finally:
        torch.randn_like = real
    assert len(zs) == 1
    z = zs[0].cpu() * 0.667
    yl = yl.cpu()
    t_y = int(yl.max())
    t_pad = 4 * math.ceil(t_y / 4)
    assert z.shape[-1] == t_pad and mel.shape[-1] == t_y
    rows = sorted(set(r % batch for r in rows) | {int(yl.argmax())})
    sd = {k: v.detach().cpu() for k, v in msd.items()}
    hp = dict(n_channels=192, n_layers=6, n_heads=2, kernel_size=3, dp_kernel_size=3, n_spks=n_spks)
    spks = sd["spk_emb.weight"][spk.cpu()[rows]] if vctk else None
    with torch.inference_mode():
        mu, logw, x_mask = O.text_encoder(O.sub(sd, "encoder"), x[rows], xl[rows], hp, spks)
        w_ceil, y_ref = O.durations(logw, x_mask)
        assert torch.equal(y_ref, yl[rows]), "duration path must be exact (forced duration head)"
        y_mask = O.sequence_mask(y_ref, t_pad).unsqueeze(1).float()
        attn = O.generate_path(w_ceil.squeeze(1), (x_mask.unsqueeze(-1) * y_mask.unsqueeze(2)).squeeze(1))
        mu_y = torch.matmul(attn.transpose(1, 2), mu.transpose(1, 2)).transpose(1, 2)
        zr = O.cfm_solve(O.sub(sd, "decoder.estimator"), mu_y, y_mask, n_ts, z[rows], spks, solver)
        mel_ref = O.denormalize(zr, sd["mel_mean"], sd["mel_std"])[:, :, :t_y]
        gs = {k: v.detach().cpu() for k, v in gsd.items()}
        bias = O.denoiser_bias_spec(gs, v1)
        # the reference's vocoder + denoiser calls are per utterance, on the mel cropped to its y_length
        # (main.py:198, MOS_audiou_generator.ipynb:276-277); the bench step does that for the batch (ragged)
        den_ref = []
        for i in range(len(rows)):
            n = int(y_ref[i])
            w = O.generator_forward(gs, mel_ref[i:i + 1, :, :n], v1).clamp(-1, 1)
            den_ref.append(O.denoise(w.squeeze(1), bias, 0.00025)[0])
    mean, std = float(sd["mel_mean"]), float(sd["mel_std"])
    mel_r = mel.cpu()[rows]
    e_mel = rel_rms((mel_r - mean) / std, (mel_ref - mean) / std)
    wav_c = wav.cpu()
    e_wav = rel_rms(torch.cat([wav_c[r, :int(yl[r]) * 256] for r in rows]), torch.cat(den_ref))
    print(f"bench step {'vctk' if vctk else 'lj'} B={batch} n={n_ts} rows {rows}: mel rel-RMS {e_mel:.3e}, "
          f"denoised wav rel-RMS {e_wav:.3e}")
    for i, r in enumerate(rows):  # every row inside its useful length (silence-free), and zero past it
        n = int(yl[r]) * 256
        assert den_ref[i].shape[0] == n
        e_row = rel_rms(wav_c[r, :n], den_ref[i])
        print(f"  row {r}: {n // 256} frames, denoised wav rel-RMS {e_row:.3e}")
        assert e_row < row_bar, (r, e_row)
        assert torch.count_nonzero(wav_c[r, n:]) == 0
    assert e_mel < 1e-2 and e_wav < 1e-2, (e_mel, e_wav)
    return t_pad


def test_bench_step_rows_vs_oracle_b32():
    """BASELINE configs[1]: the bench's own workload, rows first / middle / last / longest."""
    _bench_rows_vs_oracle(32, [0, 13, 31], "bench32")


def test_bench_step_rows_vs_oracle_b256():
    """The north-star point (B=256 on one GPU): same check on rows across the whole batch."""
    _bench_rows_vs_oracle(256, [0, 129, 255], "bench256")


def test_bench_shard_parity_rank1_of_2():
    """Multi-GPU per-shard parity: rank 1 of a world-2 bench job synthesises
    utterances [32, 64) of the global set at ITS OWN padded length with its own noise seed; those rows equal the
    oracle run on the same utterances at that T_pad. Results depend only on the shard, never on the other rank
    (no data-path collective), so this is the whole multi-GPU parity claim; rank 0 is the B=32 test above."""
    t1 = _bench_rows_vs_oracle(32, [1, 17, 30], "bench32_rank1", rank=1, world=2)
    bench = _bench()
    _, xl0 = bench.shard_inputs(0, 2, 32, 1234)
    _, xl1 = bench.shard_inputs(1, 2, 32, 1234)
    assert not torch.equal(xl0, xl1) and t1 % 4 == 0


def test_bench_step_rows_vs_oracle_vctk_config4():
    """BASELINE configs[3] per GPU: VCTK 109-speaker model with the speaker-embedding condition (the encoder and
    the estimator both read spks), 16 utterances (= 128 over 8 GPUs), 20 ODE steps, bench step rows vs oracle."""
    _bench_rows_vs_oracle(16, [0, 7, 15], "bench_vctk16", vctk=True, n_ts=20)


def test_bench_step_midpoint_solver_rows_vs_oracle():
    """The CFM's other solver (model.py:1096-1101, 'midpoint') at the bench's batch: 5 midpoint steps = the bench's
    10 estimator evaluations, bf16, rows against the oracle's midpoint solve at the bench bars."""
    _bench_rows_vs_oracle(32, [0, 13, 31], "bench32_midpoint", n_ts=5, solver="midpoint")


def test_bench_step_long_utterance_vs_oracle():
    """Size edge: a 600-phoneme utterance (1,800 mel frames with the forced duration head, 460,800 samples, about
    21 s of audio) batched with a 40-phoneme one (120 frames: 93 % of its row is padding; the batch takes the general
    attention, its first row being unpadded), through the bench step (10 ODE steps), against the oracle: the mel and
    the pair's denoised waveform at the §8c bar (1e-2; measured 5.1e-3 / 9.7e-3), each row's waveform at 1.1e-2
    (measured 9.66e-3 for the long row, 1.05e-2 for the short one: 30,720 samples, whose RMS ratio scatters more than
    the bench rows' 9.46-9.51e-3 around the bf16 path's ~9.5e-3 waveform error, DESIGN §2's error budget)."""
    g = torch.Generator().manual_seed(77)
    x = torch.randint(1, 178, (2, 600), generator=g)
    xl = torch.tensor([600, 40])
    x[1, 40:] = 0
    t_pad = _bench_rows_vs_oracle(2, [0, 1], "bench_long", n_ts=10, inputs=(x, xl), row_bar=1.1e-2)
    assert t_pad == 1800


# ------------------------------------------------------------------------------- (d) fp32 10 steps
def test_cfm_fp32_ten_steps_vs_oracle():
    from oracle import matcha_oracle as O
    dec = make_decoder(160, "fp32")
    sd = _synth_sd(dec, 12)
    dec.load_state_dict(sd)
    dec = dec.to(DEV).eval()
    B, T = 3, 240
    g = torch.Generator().manual_seed(3)
    mu = torch.randn(B, 80, T, generator=g)
    mask = (torch.arange(T)[None] < torch.tensor([240, 187, 61])[:, None]).float()[:, None]
    z = torch.randn(B, 80, T, generator=g)
    out = dec.engine().solve(dec.packed(DEV), z.to(DEV), 0.667, (mu * mask).to(DEV), mask.to(DEV), None, 10,
                             "euler").cpu()
    ref = O.cfm_solve(sd, mu * mask, mask, 10, z * 0.667)
    err = (out - ref).abs().max().item()
    print(f"fp32 10-step CFM: max|d| {err:.3e}")
    assert err < 2e-4, err


# ------------------------------------------------------------------------------- coverage
def test_every_bench_vconv_variant_was_parity_checked():
    """Each (epilogue, tile rows, tile frames, pipeline, taps) variant the bench step launches ran in
    a WHOLE-BATCH parity test above (estimator, encoder, generator), with a multi-tile grid whenever
    the bench runs it multi-tile (the bench steps themselves are only row-checked)."""
    whole = ("decoder32", "decoder128", "encoder32_fp32", "encoder256_fp32", "encoder32_bf16", "encoder256_bf16",
             "generator")
    if any(k not in LOGS for k in whole + ("bench32", "bench256")):
        pytest.skip("needs the whole module's run")
    checked = {}
    for k in whole:
        for r in LOGS[k]:
            v = _variant(r)
            checked[v] = checked.get(v, False) or r["ntiles"] > r["grid"]
    missing, single = [], []
    for r in LOGS["bench32"] + LOGS["bench256"]:
        v = _variant(r)
        if v not in checked:
            missing.append(v)
        elif r["ntiles"] > r["grid"] and not checked[v]:
            single.append(v)
    assert not missing and not single, (missing, single)
