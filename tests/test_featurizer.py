"""§8f rank 4: the log-mel featurizer (train_standalone.py:164-210 / hifigan/meldataset.py:52-89).

CPU: the product's Slaney filterbank (hifigan/meldataset.librosa_mel_fn, vectorised) against the oracle's
element-wise restatement of librosa.filters.mel, and both against an INDEPENDENT implementation of the same
published algorithm that this image carries: transformers.audio_utils.mel_filter_bank (transformers 5.15.0,
norm="slaney", mel_scale="slaney"; its own test suite checks it against librosa). librosa itself is not
installed and the reference holds no filterbank or mel output, so this is the filterbank's pin: agreement to
float32 rounding (measured ≤ 1.1e-7 relative on every nonzero weight, ≤ 1.6e-9 absolute) at the reference's
configuration and three others. The filterbank's published properties are checked too, and the oracle's framing
against an independent numpy rfft. GPU: the one-launch HIP featurizer against the oracle, atol 1e-4 on log-mel
(fp32)."""
import math

import numpy as np
import pytest
import torch

from hifigan.meldataset import librosa_mel_fn, mel_spectrogram
from oracle import matcha_oracle as O

SR, NFFT, HOP, NMEL, FMIN, FMAX = 22050, 1024, 256, 80, 0.0, 8000.0


def test_filterbank_matches_elementwise_restatement():
    a = librosa_mel_fn(SR, NFFT, NMEL, FMIN, FMAX)
    b = O.librosa_mel_basis(SR, NFFT, NMEL, FMIN, FMAX).numpy()
    assert a.shape == (80, 513) and a.dtype == np.float32
    assert np.abs(a - b).max() <= 2e-9, np.abs(a - b).max()


@pytest.mark.parametrize("sr,n_fft,n_mels,fmin,fmax", [(SR, NFFT, NMEL, FMIN, FMAX), (22050, 1024, 80, 0.0, 11025.0),
                                                    (16000, 512, 64, 20.0, 7600.0), (24000, 2048, 100, 0.0, 12000.0)])
def test_filterbank_matches_independent_implementation(sr, n_fft, n_mels, fmin, fmax):
    """Pins librosa.filters.mel(htk=False, norm="slaney") (hifigan/meldataset.py:60) without librosa: the oracle and
    the product against transformers' mel_filter_bank (float64), each weight to float32 rounding."""
    audio_utils = pytest.importorskip("transformers.audio_utils")
    ref = audio_utils.mel_filter_bank(num_frequency_bins=n_fft // 2 + 1, num_mel_filters=n_mels, min_frequency=fmin,
                                      max_frequency=fmax, sampling_rate=sr, norm="slaney", mel_scale="slaney").T
    for got in (O.librosa_mel_basis(sr, n_fft, n_mels, fmin, fmax).numpy(), librosa_mel_fn(sr, n_fft, n_mels, fmin, fmax)):
        assert got.shape == ref.shape
        d = np.abs(got.astype(np.float64) - ref)
        nz = ref > 1e-9
        assert np.all(got[~nz] == 0) or d[~nz].max() <= 1e-12
        assert (d[nz] / ref[nz]).max() <= 2.5e-7 and d.max() <= 5e-9, ((d[nz] / ref[nz]).max(), d.max())


def test_filterbank_properties():
    """Slaney filters: triangular with unit area in Hz (peak 2 / bandwidth; the 513-bin sampling of a
    triangle leaves each within 6 %, their mean within 0.1 %), peaks in increasing order, nothing above fmax,
    one contiguous support per filter."""
    w = librosa_mel_fn(SR, NFFT, NMEL, FMIN, FMAX).astype(np.float64)
    df = SR / NFFT
    area = w.sum(1) * df
    assert np.all(np.abs(area - 1) < 0.06) and abs(area.mean() - 1) < 1e-3, area
    peaks = w.argmax(1)
    assert np.all(np.diff(peaks) >= 0) and peaks[-1] * df < FMAX
    assert np.all(w[:, int(math.ceil(FMAX / df)) + 1:] == 0)
    for m in range(NMEL):  # one contiguous non-zero run per filter
        nz = np.flatnonzero(w[m])
        assert nz.size and np.all(np.diff(nz) == 1)


def test_oracle_framing_matches_numpy_rfft():
    g = np.random.RandomState(0)
    y = (g.rand(2, 5000).astype(np.float32) * 2 - 1) * 0.5
    basis = O.librosa_mel_basis(SR, NFFT, NMEL, FMIN, FMAX)
    ref = O.mel_spectrogram(torch.from_numpy(y), basis).numpy()
    p = (NFFT - HOP) // 2
    yp = np.pad(y.astype(np.float64), ((0, 0), (p, p)), mode="reflect")
    nfr = (yp.shape[1] - NFFT) // HOP + 1
    win = np.sin(np.pi * np.arange(NFFT) / NFFT) ** 2
    frames = np.stack([yp[:, f * HOP:f * HOP + NFFT] * win for f in range(nfr)], axis=-1)  # [B, n, F]
    spec = np.fft.rfft(frames, axis=1)
    mag = np.sqrt(np.abs(spec) ** 2 + 1e-9)
    mine = np.log(np.maximum(np.einsum("mk,bkf->bmf", basis.numpy().astype(np.float64), mag), 1e-5))
    assert ref.shape == (2, 80, (5000 - 256) // 256 + 1)
    assert np.abs(ref - mine).max() < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("L", [385, 22050 + 123, 3 * 22050])
def test_hip_log_mel_matches_oracle(L):
    g = torch.Generator().manual_seed(L)
    y = (torch.rand(3, L, generator=g) * 2 - 1) * torch.linspace(0.01, 0.9, 3)[:, None]
    basis = O.librosa_mel_basis(SR, NFFT, NMEL, FMIN, FMAX)
    ref = O.mel_spectrogram(y, basis)
    out = mel_spectrogram(y.cuda(), NFFT, NMEL, SR, HOP, 1024, FMIN, FMAX, center=False).cpu()
    assert out.shape == ref.shape
    err = (out - ref).abs().max().item()
    assert err < 1e-4, err
    # normalisation fused (train_standalone.py:204-210, LJSpeech statistics :802-805)
    outn = mel_spectrogram(y.cuda(), NFFT, NMEL, SR, HOP, 1024, FMIN, FMAX, mel_mean=-5.536622,
                           mel_std=2.116101).cpu()
    assert (outn - (ref + 5.536622) / 2.116101).abs().max().item() < 1e-4


def test_meldataset_host_helpers_and_normalize():
    """The reference module's host names (hifigan/meldataset.py:13-48) and train_standalone.normalize (:204-224)."""
    import numpy as np
    import pytest
    import torch
    from hifigan import meldataset as M
    assert M.MAX_WAV_VALUE == 32768.0
    x = np.array([0.5, -2.0, 1e-7], np.float32)
    assert np.allclose(M.dynamic_range_decompression(M.dynamic_range_compression(x)), np.maximum(x, 1e-5))
    t = torch.tensor([3.0, 1e-9])
    assert torch.allclose(M.spectral_de_normalize_torch(M.spectral_normalize_torch(t)), torch.tensor([3.0, 1e-5]))
    a = np.array([0.25, -0.5, 0.1], np.float32)
    assert np.allclose(M.normalize(a), a / 0.5) and M.normalize(a).dtype == np.float32  # librosa.util.normalize
    assert np.array_equal(M.normalize(np.zeros(3, np.float32)), np.zeros(3, np.float32))
    with pytest.raises(NotImplementedError):
        M.MelDataset([], 8192, 1024, 80, 256, 1024, 22050, 0, 8000)
    import train_standalone as TS
    mel = torch.randn(2, 80, 5)
    assert torch.allclose(TS.normalize(mel, -5.5, 2.1), (mel + 5.5) / 2.1)
    mu, sd = [float(i) for i in range(80)], np.full(80, 2.0, np.float32)
    assert torch.allclose(TS.normalize(mel, mu, sd), (mel - torch.arange(80.0)[:, None]) / 2.0)
