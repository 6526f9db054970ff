"""Drop-in HiFi-GAN Generator (``from hifigan.models import Generator``, main.py:136).

Same module tree and state_dict keys as the reference hifigan/models.py:14-206
(weight-norm ``weight_g``/``weight_v`` before ``remove_weight_norm``, ``weight`` after),
so ``Generator(AttrDict(v1)).load_state_dict(state["generator"])`` works unchanged.
``forward`` is the HIP vocoder (matcha_hip ``mt_vocoder_forward``); the conv modules
only hold parameters. The GAN discriminators/losses (hifigan/models.py:209-368) are
training-only and outside the synthesis hot path.
"""
from __future__ import annotations

import warnings

import torch
import torch.nn as nn
from torch.nn import Conv1d, ConvTranspose1d

from matcha_hip import runtime as rt

from .xutils import get_padding

LRELU_SLOPE = 0.1


def _wn(m):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", FutureWarning)
        return torch.nn.utils.weight_norm(m)


def _unwn(m):
    if hasattr(m, "weight_g"):
        torch.nn.utils.remove_weight_norm(m)


def _folded_weight(m) -> torch.Tensor:
    """W = g * v / ||v|| (norm over all dims but 0), or the plain weight after folding."""
    if hasattr(m, "weight_g"):
        return torch._weight_norm(m.weight_v, m.weight_g, 0)
    return m.weight


class ResBlock1(nn.Module):
    """3 x [lrelu -> conv(k, d) -> lrelu -> conv(k, 1) -> + x] (hifigan/models.py:14-103)."""

    def __init__(self, h, channels, kernel_size=3, dilation=(1, 3, 5)):
        super().__init__()
        self.h = h
        self.convs1 = nn.ModuleList([
            _wn(Conv1d(channels, channels, kernel_size, 1, dilation=d, padding=get_padding(kernel_size, d)))
            for d in dilation])
        self.convs2 = nn.ModuleList([
            _wn(Conv1d(channels, channels, kernel_size, 1, dilation=1, padding=get_padding(kernel_size, 1)))
            for _ in dilation])

    def forward(self, x):
        raise RuntimeError("ResBlock1 is evaluated inside the HIP vocoder (Generator.forward)")

    def remove_weight_norm(self):
        for m in list(self.convs1) + list(self.convs2):
            _unwn(m)


class ResBlock2(nn.Module):
    """n x [lrelu -> conv(k, d) -> + x] (hifigan/models.py:106-145)."""

    def __init__(self, h, channels, kernel_size=3, dilation=(1, 3)):
        super().__init__()
        self.h = h
        self.convs = nn.ModuleList([
            _wn(Conv1d(channels, channels, kernel_size, 1, dilation=d, padding=get_padding(kernel_size, d)))
            for d in dilation])

    def forward(self, x):
        raise RuntimeError("ResBlock2 is evaluated inside the HIP vocoder (Generator.forward)")

    def remove_weight_norm(self):
        for m in self.convs:
            _unwn(m)


class Generator(nn.Module):
    """mel [B,80,T] -> wav [B,1,T*prod(upsample_rates)] (hifigan/models.py:148-206)."""

    def __init__(self, h, precision: str = "fp32"):
        super().__init__()
        self.h = h
        self.num_kernels = len(h.resblock_kernel_sizes)
        self.num_upsamples = len(h.upsample_rates)
        self.conv_pre = _wn(Conv1d(80, h.upsample_initial_channel, 7, 1, padding=3))
        rb = ResBlock1 if h.resblock == "1" else ResBlock2
        self.ups = nn.ModuleList()
        for i, (u, k) in enumerate(zip(h.upsample_rates, h.upsample_kernel_sizes)):
            self.ups.append(_wn(ConvTranspose1d(h.upsample_initial_channel // (2 ** i),
                                                h.upsample_initial_channel // (2 ** (i + 1)), k, u,
                                                padding=(k - u) // 2)))
        self.resblocks = nn.ModuleList()
        ch = h.upsample_initial_channel
        for i in range(len(self.ups)):
            ch = h.upsample_initial_channel // (2 ** (i + 1))
            for k, d in zip(h.resblock_kernel_sizes, h.resblock_dilation_sizes):
                self.resblocks.append(rb(h, ch, k, d))
        self.conv_post = _wn(Conv1d(ch, 1, 7, 1, padding=3))
        for m in list(self.ups) + [self.conv_post]:
            with torch.no_grad():
                m.weight_v.normal_(0.0, 0.01)
        self.precision = precision
        self._engines = {}
        self._pk = rt.PackCache()

    # ---- HIP plumbing ----
    def set_precision(self, precision: str):
        rt.dtype_code(precision)
        self.precision = precision
        return self

    def engine(self) -> rt.VocoderEngine:
        if self.precision not in self._engines:
            self._engines[self.precision] = rt.VocoderEngine(dict(self.h), self.precision)
        return self._engines[self.precision]

    def folded_state(self):
        out = {}
        for name, m in self.named_modules():
            if isinstance(m, (Conv1d, ConvTranspose1d)):
                out[name + ".weight"] = _folded_weight(m)
                out[name + ".bias"] = m.bias
        return out

    def prepare(self, device):
        """Extension: check (or pack) the weights now, e.g. while the GPU still runs the acoustic model, so that the
        next forward on `device` skips the check at its start (the same cache check, done earlier; synthesize does this
        for the estimator). Only the next forward is trusted: the weights must not change between prepare() and that
        forward (an update after it is seen from the forward after that on)."""
        self.packed(device)
        self._pk.trust_next((self.precision, str(device)))

    def packed(self, device):
        key = (self.precision, str(device))
        packed = self._pk.get(key)
        if packed is None:
            src = list(self.state_dict(keep_vars=True).values())
            packed = self._pk.put(key, src, self.engine().pack(self.folded_state, src, device))
        return packed

    def forward(self, x, lengths=None):
        """``lengths`` (extension, default None = the reference's call): int [B] mel frames per utterance of a
        padded batch. Each utterance is then vocoded at its own length, as the reference pipeline calls the
        vocoder one utterance at a time on the mel `synthesize` cropped to it (main.py:181-198,
        MOS_audiou_generator.ipynb:265-277): out[b, :, :hop * lengths[b]] equals this forward on
        x[b:b+1, :, :lengths[b]] alone, and out[b] past it is zero. One batched launch chain on the bf16 path
        (mt_vocoder_forward_ragged); otherwise one call per utterance."""
        rt.require_gpu(x, what="Generator.forward")
        x = rt.f32c(x)
        eng = self.engine()
        with torch.no_grad():
            if lengths is None:
                return eng.forward(self.packed(x.device), x)
            if eng.ragged_supported():
                B = x.shape[0]
                if B <= rt.RAGGED_MAX_BATCH:
                    return eng.forward(self.packed(x.device), x, lengths=lengths)
                # more utterances than one ragged launch chain takes: consecutive chunks, each at the batch's T
                out = torch.empty((B, 1, x.shape[-1] * eng.hop), dtype=torch.float32, device=x.device)
                for s in range(0, B, rt.RAGGED_MAX_BATCH):
                    e = min(B, s + rt.RAGGED_MAX_BATCH)
                    eng.forward(self.packed(x.device), x[s:e].contiguous(), out=out[s:e], lengths=lengths[s:e])
                return out
            B, _, T = x.shape
            hop = eng.hop
            out = torch.zeros((B, 1, T * hop), dtype=torch.float32, device=x.device)
            for b, n in enumerate(int(v) for v in lengths.cpu()):
                n = max(0, min(n, T))
                if n:
                    out[b:b + 1, :, :n * hop] = eng.forward(self.packed(x.device), x[b:b + 1, :, :n].contiguous())
            return out

    def remove_weight_norm(self):
        print("Removing weight norm...")
        for m in self.ups:
            _unwn(m)
        for m in self.resblocks:
            m.remove_weight_norm()
        _unwn(self.conv_pre)
        _unwn(self.conv_post)
