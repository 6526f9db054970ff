"""Deterministic synthetic weights and inputs (no checkpoints exist offline).

Recipe: every tensor of a state dict is drawn from its
own ``numpy.random.RandomState(seed ^ crc32(key))`` so a tensor depends only on
(seed, key, shape) — the same on every machine, with or without the reference.

* conv / linear weights (ndim >= 2) and weight-norm ``weight_v``: N(0, 1/fan_in)
  (ConvTranspose1d: fan_in = C_in * k / stride, the taps one output sees)
* weight-norm ``weight_g``: ||v|| * U(0.8, 1.2) (so the fold is non-trivial)
* norm scales (1-D ``weight`` / ``gamma``): 1 + 0.1 N
* biases / ``beta`` of norms: 0.1 N
* SnakeBeta ``alpha`` / ``beta`` (log-scale): 0.2 N
* ``emb.weight``: N(0, n_channels^-0.5) (model.py:472)
* ``mel_mean`` / ``mel_std``: LJSpeech stats (train_standalone.py:802-805)
* HiFi-GAN ``conv_post``: v scaled by 0.25 so tanh is not saturated

Only numpy is needed; importing this module never touches the GPU library.
"""
from __future__ import annotations

import zlib
from typing import Dict, Iterable, Optional, Tuple

import numpy as np

LJ_MEL_MEAN = -5.536622
LJ_MEL_STD = 2.116101

_CONVT_STRIDE_HINTS = {  # key prefix -> stride for ConvTranspose1d weights
    "ups.0.": 8, "ups.1.": 8, "ups.2.": 2, "ups.3.": 2,
}


def _rs(seed: int, key: str) -> np.random.RandomState:
    return np.random.RandomState((seed ^ zlib.crc32(key.encode())) & 0x7FFFFFFF)


def _is_convt(key: str) -> Optional[int]:
    if ".up_blocks." in key and key.endswith(".2.conv.weight"):
        return 2
    for p, s in _CONVT_STRIDE_HINTS.items():
        if key.startswith(p) or ("." + p) in key:
            return s
    return None


def make_tensor(key: str, shape: Tuple[int, ...], seed: int) -> np.ndarray:
    rs = _rs(seed, key)
    shape = tuple(int(s) for s in shape)
    leaf = key.rsplit(".", 1)[-1]
    if key.endswith("mel_mean"):
        return np.full(shape, LJ_MEL_MEAN, np.float32)
    if key.endswith("mel_std"):
        return np.full(shape, LJ_MEL_STD, np.float32)
    if key.endswith("emb.weight") and len(shape) == 2 and "spk_emb" not in key:
        return (rs.standard_normal(shape) * shape[1] ** -0.5).astype(np.float32)
    if leaf in ("alpha", "beta") and "ff.net.0" in key:
        return (0.2 * rs.standard_normal(shape)).astype(np.float32)
    if leaf == "weight_g":
        # filled in by make_state_dict from the matching weight_v
        return (rs.uniform(0.8, 1.2, size=shape)).astype(np.float32)
    if leaf in ("weight", "weight_v") and len(shape) >= 2:
        s = _is_convt(key)
        if s is not None:   # [C_in, C_out, k]
            fan_in = shape[0] * shape[2] / s
        else:
            fan_in = int(np.prod(shape[1:]))
        w = rs.standard_normal(shape) / np.sqrt(fan_in)
        if key.startswith("conv_post.") or ".conv_post." in key:
            w = w * 0.25
        return w.astype(np.float32)
    if leaf in ("weight", "gamma") and len(shape) == 1:
        return (1.0 + 0.1 * rs.standard_normal(shape)).astype(np.float32)
    if leaf in ("bias", "beta"):
        return (0.1 * rs.standard_normal(shape)).astype(np.float32)
    return (0.1 * rs.standard_normal(shape)).astype(np.float32)


def make_state_dict(shapes: Iterable[Tuple[str, Tuple[int, ...]]], seed: int = 1234,
                    force_log_duration: Optional[float] = None) -> Dict[str, np.ndarray]:
    """Build a full synthetic state dict from (key, shape) pairs.

    ``force_log_duration``: set the duration predictor's final 1x1 conv to
    weight 0 / bias = value, so every token gets ceil(exp(value)) frames
    (ln 2.5 -> 3 frames/token, LJSpeech-like lengths).
    """
    shapes = sorted((k, tuple(s)) for k, s in shapes)
    out = {k: make_tensor(k, s, seed) for k, s in shapes}
    for k in list(out):
        if k.endswith(".weight_g"):
            v = out[k[: -len("_g")] + "_v"]
            n = np.sqrt((v.astype(np.float64) ** 2).sum(axis=tuple(range(1, v.ndim)), keepdims=True))
            out[k] = (n * out[k].astype(np.float64)).astype(np.float32).reshape(out[k].shape)
    if force_log_duration is not None:
        for k in out:
            if k.endswith("proj_w.proj.weight"):
                out[k] = np.zeros_like(out[k])
            if k.endswith("proj_w.proj.bias"):
                out[k] = np.full_like(out[k], force_log_duration)
    return out


def ljspeech_lengths(n: int, seed: int = 0, mean: float = 566.0, std: float = 150.0,
                     lo: int = 96, hi: int = 868) -> np.ndarray:
    """SURVEY.md §8d input R: y_len = clip(round(N(566,150)), 96, 868)."""
    rs = np.random.RandomState(seed)
    return np.clip(np.round(rs.normal(mean, std, size=n)), lo, hi).astype(np.int64)


def synthetic_text(batch: int, seed: int = 0, lo: int = 150, hi: int = 251, n_vocab: int = 178):
    """SURVEY.md §8d text->wav input: x_len ~ U[lo,hi], ids ~ U[1,n_vocab-1] at odd
    positions and blank 0 at even positions (main.py:52-55 intersperse)."""
    rs = np.random.RandomState(seed)
    lens = rs.randint(lo, hi + 1, size=batch).astype(np.int64)
    tmax = int(lens.max())
    x = np.zeros((batch, tmax), np.int64)
    for b, L in enumerate(lens):
        ids = rs.randint(1, n_vocab, size=L)
        ids[0::2] = 0
        x[b, :L] = ids
    return x, lens
