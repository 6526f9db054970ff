"""bf16 performance mode: where the error comes from, and the exact index path (MI355X).

SURVEY.md §8c sets the bf16 bar at rel-RMS <= 1e-2 against fp32 (the reference under autocast-bf16 drifts
~3e-3). These tests localise the estimator's error block by block with the debug taps of
``mt_decoder_set_taps`` against
  * the reference's own forward-hook outputs in fixture G2 (tests/golden/make_golden.py:130-137), and
  * the oracle's taps at the bench shape (B=32, T=728),
and pin the index path of the bf16 model on UNFORCED synthetic duration weights: the text encoder and duration
predictor run in fp32 in the bf16 mode (model.MatchaTTS docstring), so y_lengths and attn must be bit-exact
against the oracle on non-degenerate logw (model.py:1273-1289).
Reference: model.py:964-1048 (Decoder.forward), 777-790 (ResnetBlock1D), 733-744 (BasicTransformerBlock).
"""
import math

import numpy as np
import pytest
import torch

from conftest import golden, make_decoder, make_matcha, rel_rms, t, weights_from

pytestmark = pytest.mark.gpu
DEV = "cuda"
TAPS = ("down0_res", "down0_tb", "mid1_tb", "up0_out", "up1_tb")
BF16_BAR = 1e-2


def _masked(x, mask):
    """x [B,C,T_l] * the mask at x's resolution (mask[:, :, ::2] at T/2, model.py:1006)"""
    m = mask if mask.shape[-1] == x.shape[-1] else mask[:, :, ::2]
    return x * m


def _tap_errors(taps, ref, mask):
    return {k: rel_rms(_masked(taps[k].cpu(), mask), _masked(ref[k], mask)) for k in TAPS}


def test_decoder_bf16_taps_vs_reference_hooks_g2():
    """One bf16 estimator evaluation on fixture G2 (LJ, B=2, T=64, row 1 padded): every tapped block output
    against the REFERENCE's forward-hook outputs, over the valid frames."""
    g = golden("g2_decoder_lj")
    sd = weights_from(g)
    dec = make_decoder(160, "bf16")
    dec.load_state_dict(sd)
    dec = dec.to(DEV).eval()
    x, mask, mu = t(g["x"]), t(g["mask"]), t(g["mu"])
    eng = dec.engine()
    out, taps = eng.step_taps(dec.packed(DEV), x.to(DEV), mu.to(DEV), mask.to(DEV), None, float(g["t0"]))
    ref = {k: t(g[k]) for k in TAPS}
    for k in ("down0_tb", "mid1_tb", "up1_tb"):  # the hooks saw b t c inside the rearranged block
        ref[k] = ref[k].transpose(1, 2)
    errs = _tap_errors(taps, ref, mask)
    errs["out"] = rel_rms(out.cpu(), t(g["out_t0"]))
    print("G2 bf16 rel-RMS by block: " + ", ".join(f"{k} {v:.2e}" for k, v in errs.items()))
    assert all(v < BF16_BAR for v in errs.values()), errs


@pytest.mark.parametrize("B", [32])
def test_decoder_bf16_taps_bench_shape_vs_oracle(B):
    """The same taps at the bench shape (B=32, T=728, LJSpeech-shaped ragged lengths, one unpadded row) against
    the oracle's taps (oracle.decoder_forward(taps=...), pinned to the reference's hooks by test_oracle_golden)."""
    from oracle import matcha_oracle as O
    from matcha_hip import synthetic
    dec = make_decoder(160, "bf16")
    sd = {k: torch.from_numpy(v) for k, v in synthetic.make_state_dict(
        [(k, tuple(v.shape)) for k, v in dec.state_dict().items()], 5).items()}
    dec.load_state_dict(sd)
    dec = dec.to(DEV).eval()
    T = 728
    rs = np.random.RandomState(B)
    lens = np.clip(np.round(rs.normal(566, 150, B)), 96, T).astype(np.int64)
    lens[0] = T
    gen = torch.Generator().manual_seed(B)
    x, mu = torch.randn(B, 80, T, generator=gen) * 0.667, torch.randn(B, 80, T, generator=gen)
    mask = (torch.arange(T)[None] < torch.from_numpy(lens)[:, None]).float()[:, None]
    out, taps = dec.engine().step_taps(dec.packed(DEV), x.to(DEV), (mu * mask).to(DEV), mask.to(DEV), None, 0.3)
    ref = {}
    ref_out = O.decoder_forward(sd, x, mask, mu * mask, torch.full((B,), 0.3), taps=ref)
    errs = _tap_errors(taps, ref, mask)
    errs["out"] = rel_rms(out.cpu(), ref_out)
    print(f"B={B} T={T} bf16 rel-RMS by block: " + ", ".join(f"{k} {v:.2e}" for k, v in errs.items()))
    # the reference's own bf16 mode (torch.autocast over the same ops, SURVEY.md §7 'Dtype') on the same inputs
    ac = {}
    with torch.inference_mode(), torch.autocast("cpu", dtype=torch.bfloat16):
        ac_out = O.decoder_forward(sd, x, mask, mu * mask, torch.full((B,), 0.3), taps=ac)
    ac_errs = _tap_errors({k: v.float() for k, v in ac.items()}, ref, mask)
    ac_errs["out"] = rel_rms(ac_out.float(), ref_out)
    print(f"B={B} T={T} reference autocast-bf16 rel-RMS by block: "
          + ", ".join(f"{k} {v:.2e}" for k, v in ac_errs.items()))
    assert all(v < BF16_BAR for v in errs.values()), errs
    assert errs["out"] <= ac_errs["out"], (errs["out"], ac_errs["out"])


@pytest.mark.parametrize("B,T", [(2, 160), (1, 728)])
def test_generator_bf16_no_worse_than_reference_autocast(B, T):
    """HiFi-GAN in bf16 against the fp32 oracle, next to the reference's own autocast-bf16 on the same weights and
    mel (B=2, T=160, and one bench-length utterance, T=728 mel frames = 186k samples through every stage at full
    tile counts): the HIP path's drift stays within the §8c bar and at or below autocast's."""
    from hifigan.config import v1
    from matcha_hip import synthetic
    from oracle import matcha_oracle as O
    from conftest import make_generator
    gen = make_generator("bf16")
    gen.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_state_dict(
        [(k, tuple(v.shape)) for k, v in gen.state_dict().items()], 8).items()})
    gen = gen.to(DEV).eval()
    gen.remove_weight_norm()
    gs = {k: v.cpu() for k, v in gen.state_dict().items()}
    mel = torch.randn(B, 80, T, generator=torch.Generator().manual_seed(9)) * 2.1 - 5.5
    wav = gen(mel.to(DEV)).cpu()
    with torch.inference_mode():
        ref = O.generator_forward(gs, mel, v1)
        with torch.autocast("cpu", dtype=torch.bfloat16):
            ac = O.generator_forward(gs, mel, v1).float()
    e, e_ac = rel_rms(wav, ref), rel_rms(ac, ref)
    print(f"generator bf16 rel-RMS {e:.2e}; reference autocast-bf16 {e_ac:.2e}")
    assert e < BF16_BAR and e <= e_ac, (e, e_ac)


def test_bf16_model_index_path_bit_exact_unforced_durations():
    """The bench's text batch (B=32, x_len ~ U[150,251]) through the bf16 model with UNFORCED synthetic
    duration-predictor weights: y_lengths and the alignment are bit-exact against the oracle's durations and
    generate_path on the oracle encoder's logw (model.py:1273-1289; the encoder runs fp32 in the bf16 mode)."""
    from matcha_hip import runtime as rt
    from matcha_hip import synthetic
    from oracle import matcha_oracle as O
    m = make_matcha(1, precision="bf16")
    assert m.encoder.precision == "fp32"
    sd = {k: torch.from_numpy(v) for k, v in synthetic.make_state_dict(
        [(k, tuple(v.shape)) for k, v in m.state_dict().items()], 77).items()}
    assert float(sd["encoder.proj_w.proj.weight"].abs().sum()) > 0  # a real (not forced) duration head
    m.load_state_dict(sd)
    m = m.to(DEV).eval()
    x, xl = synthetic.synthetic_text(32, seed=1234)
    x, xl = torch.from_numpy(x)[:, : int(xl.max())], torch.from_numpy(xl)
    x = x.contiguous()
    with torch.inference_mode():
        mu, logw, xm = m.encoder(x.to(DEV), xl.to(DEV))
        w_ceil, cum, yl = rt.durations(logw, xm, 1.0)
    hp = dict(n_channels=192, n_layers=6, n_heads=2, kernel_size=3, dp_kernel_size=3, n_spks=1)
    esd = {k[len("encoder."):]: v for k, v in sd.items() if k.startswith("encoder.")}
    mu_o, logw_o, xm_o = O.text_encoder(esd, x, xl, hp)
    e_logw = (logw.cpu() - logw_o).abs().max().item()
    e_mu = rel_rms(mu.cpu(), mu_o)
    wc_o, yl_o = O.durations(logw_o, xm_o)
    print(f"unforced durations B=32: logw max|d| {e_logw:.2e}, mu rel-RMS {e_mu:.2e}, "
          f"y_lengths {int(yl_o.min())}..{int(yl_o.max())}")
    assert torch.equal(xm.cpu(), xm_o)
    assert e_logw < 1e-4 and e_mu < 1e-4, (e_logw, e_mu)
    assert torch.equal(yl.cpu(), yl_o), "y_lengths must be bit-exact"
    assert torch.equal(w_ceil.cpu(), wc_o)
    # the whole synthesize call: lengths and the alignment exact, mel within the bf16 bar (2 ODE steps)
    torch.manual_seed(5)
    zs = []
    real = torch.randn_like

    def noise(ref_, *a, **k):
        zs.append(real(ref_))
        return zs[-1].clone()

    torch.randn_like = noise
    try:
        mel, yl2, attn = m.synthesize(x.to(DEV), xl.to(DEV), n_timesteps=2, temperature=0.667)
    finally:
        torch.randn_like = real
    t_y = int(yl_o.max())
    t_pad = 4 * math.ceil(t_y / 4)
    y_mask = O.sequence_mask(yl_o, t_pad).unsqueeze(1).float()
    attn_o = O.generate_path(wc_o.squeeze(1), (xm_o.unsqueeze(-1) * y_mask.unsqueeze(2)).squeeze(1))
    assert torch.equal(yl2.cpu(), yl_o)
    assert torch.equal(attn.cpu().squeeze(1), attn_o), "alignment must be bit-exact"
    rows = [0, 15, 31]
    mu_y = torch.matmul(attn_o.transpose(1, 2), mu_o.transpose(1, 2)).transpose(1, 2)[rows]
    zr = O.cfm_solve(O.sub(sd, "decoder.estimator"), mu_y, y_mask[rows], 2, zs[0].cpu()[rows] * 0.667)
    mel_o = O.denormalize(zr, sd["mel_mean"], sd["mel_std"])[:, :, :t_y]
    mean, std = float(sd["mel_mean"]), float(sd["mel_std"])
    e_mel = rel_rms((mel.cpu()[rows] - mean) / std, (mel_o - mean) / std)
    print(f"unforced durations B=32: T_pad {t_pad}, mel rel-RMS (rows {rows}) {e_mel:.2e}")
    assert e_mel < BF16_BAR, e_mel
