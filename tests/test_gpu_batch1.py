"""Batch 1 on the HIP path: BASELINE configs[0]'s workload (1 utterance, 4 Euler steps) and the published comparison
point's (batch-1 text->wav + denoiser at 10 steps, MOS_audiou_generator.ipynb:257), against the oracle (MI355X).

At batch 1 the padded length T_pad = 4*ceil(y_len/4) (model.py:1281) decides the decoder's attention path:
y_len % 4 != 0 leaves 1-3 padded frames, the reference's +3.4e38 fill (model.py:697) makes every query attend
uniformly to them and the solver takes the query-independent path; y_len % 4 == 0 leaves none and the general
Q.K^T path runs. The bench weights force 3 frames per token, so x_len 150 -> y_len 450 (padded)
and x_len 152 -> y_len 456 (unpadded) select the two paths.
Tolerances: fp32 mel atol 2e-4 (CFM), waveform atol 1e-5 (measured 2.6e-6..3.3e-6 max |d|);
bf16 rel-RMS 1e-2 on the normalised mel and on the denoised waveform.
Reference: model.py:1264-1300, hifigan/models.py:181-197, hifigan/denoiser.py:62-68.
"""
import math
import os
import sys

import pytest
import torch

from conftest import REPO, rel_rms

pytestmark = pytest.mark.gpu
DEV = "cuda"
_MODELS = {}


def _bench():
    if REPO not in sys.path:
        sys.path.insert(0, REPO)
    import bench
    return bench


def _models(precision):
    if precision not in _MODELS:
        _MODELS[precision] = _bench().build_models(torch.device(DEV), precision, 1234)
    return _MODELS[precision]


def _utterance(x_len):
    from matcha_hip import synthetic
    x, xl = synthetic.synthetic_text(1, seed=x_len, lo=x_len, hi=x_len)
    return torch.from_numpy(x), torch.from_numpy(xl)


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
@pytest.mark.parametrize("n_ts", [4, 10])
@pytest.mark.parametrize("x_len", [150, 152])
def test_batch1_text_to_wav_vs_oracle(precision, n_ts, x_len):
    from hifigan.config import v1
    from oracle import matcha_oracle as O
    bench = _bench()
    m, g, den, msd, gsd = _models(precision)
    x, xl = _utterance(x_len)
    torch.manual_seed(n_ts)
    zs = []
    real = torch.randn_like

    def noise(ref, *a, **k):
        zs.append(real(ref))
        return zs[-1].clone()

    torch.randn_like = noise
    try:
        mel, yl, wav = bench.step(m, g, den, x.to(DEV), xl.to(DEV), n_ts, True)
        torch.cuda.synchronize()
    finally:
        torch.randn_like = real
    y_len = 3 * x_len
    t_pad = 4 * math.ceil(y_len / 4)
    assert int(yl[0]) == y_len and zs[0].shape[-1] == t_pad and mel.shape[-1] == y_len
    sd = {k: v.detach().cpu() for k, v in msd.items()}
    gs = {k: v.detach().cpu() for k, v in gsd.items()}
    hp = dict(n_channels=192, n_layers=6, n_heads=2, kernel_size=3, dp_kernel_size=3, n_spks=1)
    with torch.inference_mode():
        mel_o, yl_o, _ = O.synthesize(sd, x, xl, n_ts, lambda mu: zs[0].cpu() * 0.667, hp)
        wav_o = O.generator_forward(gs, mel_o, v1).clamp(-1, 1)
        den_o = O.denoise(wav_o.squeeze(1), O.denoiser_bias_spec(gs, v1), 0.00025)
    assert torch.equal(yl.cpu(), yl_o)
    mean, std = float(sd["mel_mean"]), float(sd["mel_std"])
    path = "general attention" if y_len % 4 == 0 else "query-independent attention"
    if precision == "fp32":
        e_mel = (mel.cpu() - mel_o).abs().max().item()
        e_wav = (wav.cpu() - den_o).abs().max().item()
        print(f"B=1 fp32 n={n_ts} y_len={y_len} ({path}): mel max|d| {e_mel:.2e}, wav max|d| {e_wav:.2e}")
        assert e_mel < 2e-4 and e_wav < 1e-5, (e_mel, e_wav)  # SURVEY §8c atol 1e-5 (measured wav 2.6e-6..3.3e-6)
    else:
        e_mel = rel_rms((mel.cpu() - mean) / std, (mel_o - mean) / std)
        e_wav = rel_rms(wav.cpu(), den_o)
        print(f"B=1 bf16 n={n_ts} y_len={y_len} ({path}): mel rel-RMS {e_mel:.2e}, wav rel-RMS {e_wav:.2e}")
        assert e_mel < 1e-2 and e_wav < 1e-2, (e_mel, e_wav)
