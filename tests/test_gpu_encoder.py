"""Text encoder + duration predictor on the MI355X (mt_encoder) against the CPU
oracle (oracle/matcha_oracle.py:text_encoder, pinned to the reference by tests/golden/g6_*).

fp32 parity mode: mu / logw max-abs <= 1e-4, x_mask exact. This fp32 encoder is what BOTH model precisions run
(model.MatchaTTS: the index path is exact only on fp32 logw). The opt-in encoder_precision="bf16" mode, off the
product path, is held to the 2e-2 it was built to (measured 1.1e-2), not to the §8c contract.
Cases: LJ (single speaker) and VCTK (spk-embedding channels), ragged lengths including a length-1
utterance, Tx crossing the attention kernel's 64-key chunks, B = 1.
"""
import math

import pytest
import torch

from conftest import HP, make_matcha, rel_rms
from matcha_hip import synthetic
from oracle import matcha_oracle as O

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _model(n_spks, precision, seed):
    """precision: the TEXT ENCODER's (bf16 = the opt-in encoder_precision="bf16" mode)"""
    m = make_matcha(n_spks, precision)
    m.set_precision(precision, encoder_precision=precision)
    sd = {k: torch.from_numpy(v) for k, v in synthetic.make_state_dict(
        [(k, tuple(v.shape)) for k, v in m.state_dict().items()], seed).items()}
    m.load_state_dict(sd)
    return m.to(DEV).eval(), sd


def _inputs(lengths, seed):
    g = torch.Generator().manual_seed(seed)
    Tx = max(lengths)
    x = torch.randint(1, 178, (len(lengths), Tx), generator=g)
    xl = torch.tensor(lengths, dtype=torch.int64)
    for i, n in enumerate(lengths):
        x[i, n:] = 0
    return x, xl


CASES = [
    ("lj", 1, [37, 12, 1]),
    ("lj_chunks", 1, [130, 65, 64]),
    ("vctk", 4, [50, 23]),
    ("lj_b1", 1, [9]),
]


@pytest.mark.parametrize("name,n_spks,lengths", CASES, ids=[c[0] for c in CASES])
def test_text_encoder_fp32_matches_oracle(name, n_spks, lengths):
    m, sd = _model(n_spks, "fp32", 11 + n_spks)
    x, xl = _inputs(lengths, len(lengths) * 7 + n_spks)
    spks = torch.randn(len(lengths), 64, generator=torch.Generator().manual_seed(5)) if n_spks > 1 else None
    mu, logw, xm = m.encoder(x.to(DEV), xl.to(DEV), None if spks is None else spks.to(DEV))
    torch.cuda.synchronize()
    hp = dict(HP, n_spks=n_spks)
    sub = {k[len("encoder."):]: v for k, v in sd.items() if k.startswith("encoder.")}
    mu_o, logw_o, xm_o = O.text_encoder(sub, x, xl, hp, spks)
    assert torch.equal(xm.cpu(), xm_o)
    e_mu = (mu.cpu() - mu_o).abs().max().item()
    e_w = (logw.cpu() - logw_o).abs().max().item()
    assert e_mu < 1e-4 and e_w < 1e-4, (e_mu, e_w)


def test_text_encoder_bf16_close():
    m, sd = _model(1, "bf16", 21)
    x, xl = _inputs([80, 41, 7], 3)
    mu, logw, _ = m.encoder(x.to(DEV), xl.to(DEV))
    sub = {k[len("encoder."):]: v for k, v in sd.items() if k.startswith("encoder.")}
    mu_o, logw_o, _ = O.text_encoder(sub, x, xl, dict(HP, n_spks=1))
    assert rel_rms(mu.cpu(), mu_o) < 2e-2
    assert rel_rms(logw.cpu(), logw_o) < 2e-2


@pytest.mark.parametrize("lengths", [[80, 41, 7], [250, 193, 64, 1], [130, 129, 65]])
def test_text_encoder_bf16_mfma_attention(lengths):
    """bf16, 96-dim heads: the attention core on MFMA (enc_attn_mfma96_kernel: S^T = K.Q^T, online softmax,
    O^T = V^T.P^T with bf16 probabilities) against the fp32-VALU kernel (rel-RMS 1e-2) and the fp32 oracle
    (2e-2), over key tiles that are partly / wholly padding and query tiles past Tx."""
    m, sd = _model(1, "bf16", 29)
    x, xl = _inputs(lengths, 5)
    eng = m.encoder.engine()
    sub = {k[len("encoder."):]: v for k, v in sd.items() if k.startswith("encoder.")}
    mu_o, logw_o, _ = O.text_encoder(sub, x, xl, dict(HP, n_spks=1))
    try:
        eng.set_mfma_attention(0)
        mu_v, logw_v, _ = m.encoder(x.to(DEV), xl.to(DEV))
        eng.set_mfma_attention(1)
        mu_m, logw_m, xm = m.encoder(x.to(DEV), xl.to(DEV))
    finally:
        eng.set_mfma_attention(1)
    mu_m, mu_v, logw_m, logw_v = mu_m.cpu(), mu_v.cpu(), logw_m.cpu(), logw_v.cpu()
    assert torch.isfinite(mu_m).all() and torch.isfinite(logw_m).all()
    assert not torch.equal(mu_m, mu_v)  # the MFMA kernel ran
    e_m = (rel_rms(mu_m, mu_o), rel_rms(logw_m, logw_o))
    e_v = (rel_rms(mu_v, mu_o), rel_rms(logw_v, logw_o))
    print(f"mfma vs valu {rel_rms(mu_m, mu_v):.3e} / {rel_rms(logw_m, logw_v):.3e}; vs oracle: mfma "
          f"{e_m[0]:.3e} / {e_m[1]:.3e}, valu {e_v[0]:.3e} / {e_v[1]:.3e}")
    assert e_m[0] < 2e-2 and e_m[1] < 2e-2  # the bf16 encoder bar (test_text_encoder_bf16_close)
    # no worse than the VALU kernel beyond bf16 noise (the duration head amplifies rounding in logw)
    assert e_m[0] < 1.5 * e_v[0] + 2e-3 and e_m[1] < 1.5 * e_v[1] + 2e-3
    assert torch.equal(mu_m * xm.cpu(), mu_m)  # padded frames stay zero


def test_text_encoder_forced_duration_head_exact():
    """With the bench's forced duration head (proj weight 0, bias ln 2.5) logw is exactly
    ln(2.5) * x_mask in every precision, so the index path downstream is exact."""
    for precision in ("fp32", "bf16"):
        m = make_matcha(1, precision)
        sd = {k: torch.from_numpy(v) for k, v in synthetic.make_state_dict(
            [(k, tuple(v.shape)) for k, v in m.state_dict().items()], 3,
            force_log_duration=math.log(2.5)).items()}
        m.load_state_dict(sd)
        m = m.to(DEV).eval()
        x, xl = _inputs([40, 17], 9)
        _, logw, xm = m.encoder(x.to(DEV), xl.to(DEV))
        ref = torch.full_like(logw, math.log(2.5)) * xm
        assert torch.equal(logw, ref.to(torch.float32)), precision


@pytest.mark.parametrize("name,n_spks,lengths", CASES[:3], ids=[c[0] for c in CASES[:3]])
def test_text_encoder_fp32_vconv_matches_generic_kernel(name, n_spks, lengths):
    """fp32: the convs on mt_vconv's fp32 mode and the attention core on exact-fp32 MFMA (defaults) against the
    generic conv kernel and the VALU attention (mt_encoder_set_vconv(0), set_mfma_attention(0)) on the same inputs:
    same arithmetic, different accumulation order -> within fp32 rounding (both vs the oracle in the test above)."""
    m, sd = _model(n_spks, "fp32", 11 + n_spks)
    x, xl = _inputs(lengths, len(lengths) * 7 + n_spks)
    spks = torch.randn(len(lengths), 64, generator=torch.Generator().manual_seed(5)) if n_spks > 1 else None
    args = (x.to(DEV), xl.to(DEV), None if spks is None else spks.to(DEV))
    eng = m.encoder.engine()
    mu1, logw1, xm1 = m.encoder(*args)
    eng.set_vconv(0)
    eng.set_mfma_attention(0)
    try:
        mu0, logw0, xm0 = m.encoder(*args)
    finally:
        eng.set_vconv(1)
        eng.set_mfma_attention(1)
    assert torch.equal(xm0, xm1)
    e_mu, e_logw = (mu1 - mu0).abs().max().item(), (logw1 - logw0).abs().max().item()
    print(f"{name}: fp32 vconv vs generic: mu max|d| {e_mu:.2e}, logw max|d| {e_logw:.2e}")
    assert e_mu < 2e-5 and e_logw < 2e-5, (e_mu, e_logw)


@pytest.mark.parametrize("bad,where", [(178, "live"), (-1, "live"), (500, "padding")])
def test_out_of_vocabulary_id_raises(bad, where):
    """nn.Embedding's error semantics (model.py:471, 522: ``self.emb(x)`` raises IndexError for an id outside
    [0, n_vocab), including one in the padded tail of x): TextEncoder.forward and MatchaTTS.synthesize raise
    IndexError instead of synthesizing from a clamped row; the largest valid id (n_vocab - 1) runs, and the same
    model still synthesizes afterwards."""
    m, _ = _model(1, "fp32", 13)
    x, xl = _inputs([20, 11], 3)
    x[0, 5] = 177  # n_vocab - 1 is valid
    mu, _, _ = m.encoder(x.to(DEV), xl.to(DEV))
    assert torch.isfinite(mu).all()
    xb = x.clone()
    if where == "live":
        xb[1, 4] = bad
    else:
        xb[1, 15] = bad  # past x_lengths[1] = 11
    with pytest.raises(IndexError):
        m.encoder(xb.to(DEV), xl.to(DEV))
    with pytest.raises(IndexError):
        m.synthesize(xb.to(DEV), xl.to(DEV), n_timesteps=2, temperature=0.667)
    mel, yl, _ = m.synthesize(x.to(DEV), xl.to(DEV), n_timesteps=2, temperature=0.667)
    assert torch.isfinite(mel).all() and int(yl.min()) >= 1
