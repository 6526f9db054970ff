"""Drop-in ``hifigan.meldataset`` featurizer (§8f rank 4): ``mel_spectrogram`` as the reference's training
data path computes it (train_standalone.py:164-201 == hifigan/meldataset.py:52-89), on the MI355X.

The filterbank is librosa's Slaney mel basis (``librosa.filters.mel(sr, n_fft, n_mels, fmin, fmax)``,
htk=False, norm="slaney", float32): librosa is not a dependency here, so ``librosa_mel_fn`` restates
its published algorithm (host numpy, a constant per configuration, cached per device). The spectrogram
itself (reflect pad, STFT, magnitude, filterbank, log, normalisation) is ONE HIP launch
(``mt_log_mel``); there is no CPU fallback, so featurization runs in the main (GPU) process: the reference's
DataLoader CPU workers (train_standalone.py:408-411, num_workers=8) cannot call it.
The module's host helpers keep the reference's names (MAX_WAV_VALUE, load_wav, dynamic_range_*,
spectral_*normalize_torch, normalize = librosa.util.normalize for audio); ``MelDataset`` (HiFi-GAN GAN training
data, out of scope) raises.
"""
from __future__ import annotations

import numpy as np
import torch

from matcha_hip._lib import check, lib, stream_handle
from matcha_hip.runtime import require_gpu

MAX_WAV_VALUE = 32768.0  # hifigan/meldataset.py:13


def load_wav(full_path):
    """hifigan/meldataset.py:16-18 -> (data, sampling_rate) via scipy.io.wavfile.read"""
    from scipy.io.wavfile import read
    sampling_rate, data = read(full_path)
    return data, sampling_rate


def dynamic_range_compression(x, C=1, clip_val=1e-5):
    return np.log(np.clip(x, a_min=clip_val, a_max=None) * C)


def dynamic_range_decompression(x, C=1):
    return np.exp(x) / C


def dynamic_range_compression_torch(x, C=1, clip_val=1e-5):
    return torch.log(torch.clamp(x, min=clip_val) * C)


def dynamic_range_decompression_torch(x, C=1):
    return torch.exp(x) / C


def spectral_normalize_torch(magnitudes):
    return dynamic_range_compression_torch(magnitudes)


def spectral_de_normalize_torch(magnitudes):
    return dynamic_range_decompression_torch(magnitudes)


def normalize(S, norm=np.inf, axis=0, threshold=None, fill=None):
    """librosa.util.normalize as hifigan/meldataset.py imports it (peak-normalising audio before featurizing):
    S scaled so that its `norm` along `axis` is 1; slices whose norm is below `threshold` (default: the smallest
    positive normal of the dtype) are left unscaled (fill=None). numpy in, numpy out."""
    if fill is not None:
        raise NotImplementedError("normalize(fill=...) is not used by the reference")
    S = np.asarray(S)
    mag = np.abs(S).astype(np.float64)
    if threshold is None:
        threshold = np.finfo(S.dtype if np.issubdtype(S.dtype, np.floating) else np.float32).tiny
    if norm == np.inf:
        length = np.max(mag, axis=axis, keepdims=True)
    elif norm == -np.inf:
        length = np.min(mag, axis=axis, keepdims=True)
    elif norm == 0:
        length = np.sum(mag > 0, axis=axis, keepdims=True).astype(mag.dtype)
    else:
        length = np.sum(mag ** norm, axis=axis, keepdims=True) ** (1.0 / norm)
    length = np.where(length < threshold, 1.0, length)
    return (S / length).astype(S.dtype) if np.issubdtype(S.dtype, np.floating) else S / length


class MelDataset:
    """hifigan/meldataset.py:105-217 (the GAN vocoder's training data) is out of scope."""

    def __init__(self, *a, **k):
        raise NotImplementedError("MelDataset (HiFi-GAN GAN training data) is not part of the MI355X path; featurize "
                                  "in the main process with mel_spectrogram(...) on GPU tensors (INTEGRATION.md)")


_F_SP, _MIN_LOG_HZ = 200.0 / 3, 1000.0
_MIN_LOG_MEL = _MIN_LOG_HZ / _F_SP
_LOGSTEP = np.log(6.4) / 27.0


def _hz_to_mel(f):
    f = np.asarray(f, dtype=np.float64)
    return np.where(f >= _MIN_LOG_HZ, _MIN_LOG_MEL + np.log(np.maximum(f, 1e-300) / _MIN_LOG_HZ) / _LOGSTEP,
                    f / _F_SP)


def _mel_to_hz(m):
    m = np.asarray(m, dtype=np.float64)
    return np.where(m >= _MIN_LOG_MEL, _MIN_LOG_HZ * np.exp(_LOGSTEP * (m - _MIN_LOG_MEL)), _F_SP * m)


def librosa_mel_fn(sr, n_fft, n_mels=128, fmin=0.0, fmax=None):
    """librosa.filters.mel(sr=, n_fft=, n_mels=, fmin=, fmax=) (Slaney scale and area norm) -> [n_mels, 1+n_fft//2]
    float32: triangles between consecutive mel-spaced edge frequencies, each rounded to float32, then scaled
    by 2 / (f[i+2] - f[i]) and rounded again (librosa's in-place float32 `weights *= enorm`)."""
    fmax = float(sr) / 2 if fmax is None else float(fmax)
    fft_f = np.arange(1 + n_fft // 2, dtype=np.float64) * (float(sr) / n_fft)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(fmin), _hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = mel_f[:, None] - fft_f[None, :]
    lower = -ramps[:n_mels] / fdiff[:n_mels, None]
    upper = ramps[2:n_mels + 2] / fdiff[1:n_mels + 1, None]
    w = np.maximum(0.0, np.minimum(lower, upper)).astype(np.float32)
    enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
    return (w.astype(np.float64) * enorm[:, None]).astype(np.float32)


_BASIS = {}


def mel_spectrogram(y, n_fft, num_mels, sampling_rate, hop_size, win_size, fmin, fmax, center=False,
                    mel_mean=0.0, mel_std=1.0):
    """train_standalone.py:164-201 on the GPU: y [B, L] (or [L]) fp32 in [-1, 1] -> log-mel [B, num_mels, F],
    F = (L - 256) // 256 + 1; with mel_mean / mel_std also `normalize` (train_standalone.py:204-210), fused.
    Built for the reference's configuration (n_fft = win = 1024, hop = 256, 80 mels, center=False)."""
    if (n_fft, win_size, hop_size, num_mels, bool(center)) != (1024, 1024, 256, 80, False):
        raise NotImplementedError("the HIP featurizer is built for n_fft=win=1024, hop=256, 80 mels, center=False "
                                  "(train_standalone.py:819-827)")
    require_gpu(y, what="mel_spectrogram")
    y = y.detach().to(torch.float32)
    squeeze = y.dim() == 1
    y = y.reshape(1, -1) if squeeze else y.reshape(y.shape[0], -1)
    y = y.contiguous()
    B, L = y.shape
    if L <= 384:
        raise ValueError(f"mel_spectrogram: {L} samples; reflect padding needs more than 384")
    key = (sampling_rate, n_fft, num_mels, float(fmin), float(fmax), str(y.device))
    basis = _BASIS.get(key)
    if basis is None:
        basis = torch.from_numpy(librosa_mel_fn(sampling_rate, n_fft, num_mels, fmin, fmax)).to(y.device)
        _BASIS[key] = basis
    F = (L - 256) // 256 + 1
    out = torch.empty((B, num_mels, F), dtype=torch.float32, device=y.device)
    check(lib().mt_log_mel(y.data_ptr(), B, L, basis.data_ptr(), float(mel_mean), float(mel_std), out.data_ptr(),
                           stream_handle(y.device)), "log_mel")
    return out[0] if squeeze else out

