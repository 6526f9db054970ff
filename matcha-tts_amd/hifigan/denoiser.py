"""Drop-in Denoiser (hifigan/denoiser.py:11-68): removes the vocoder's bias spectrum.

bias_spec = |STFT(vocoder(zeros[1,80,88]))| of frame 0 (mode "zeros"), computed with the
HIP STFT kernel; forward(audio [B,L], strength) runs the fused HIP
STFT -> clamp(|S| - strength*bias, 0) -> iSTFT path (mt_denoise).
"""
from __future__ import annotations

import torch

from matcha_hip import runtime as rt


class ModeException(Exception):
    pass


class Denoiser(torch.nn.Module):
    def __init__(self, vocoder, filter_length=1024, n_overlap=4, win_length=1024, mode="zeros"):
        super().__init__()
        if filter_length != 1024 or n_overlap != 4 or win_length != 1024:
            raise NotImplementedError("the HIP denoiser implements n_fft=1024, hop=256, win=1024")
        self.filter_length = filter_length
        self.hop_length = int(filter_length / n_overlap)
        self.win_length = win_length
        p = next(vocoder.parameters())
        self.device = p.device
        if mode == "zeros":
            mel = torch.zeros((1, 80, 88), dtype=p.dtype, device=p.device)
        elif mode == "normal":
            mel = torch.randn((1, 80, 88), dtype=p.dtype, device=p.device)
        else:
            raise ModeException(f"Mode {mode} if not supported")
        with torch.no_grad():
            bias_audio = vocoder(mel).float().squeeze(0)          # [1, L]
            mag = rt.stft_magnitude(bias_audio)                  # [1, frames, 513]
        self.register_buffer("bias_spec", mag[:, 0, :][:, :, None].contiguous())  # [1, 513, 1]

    @torch.inference_mode()
    def forward(self, audio, strength=0.0005, lengths=None):
        """``lengths`` (extension, default None = the reference's call): int [B] utterance lengths in units of 256
        samples (mel frames) for a padded [B, L] batch; row b is then denoised as the one-utterance call on its
        first 256 * lengths[b] samples (its own reflect padding and frame count) and is zero past them."""
        squeeze = audio.dim() == 1
        a = audio.unsqueeze(0) if squeeze else audio
        out = rt.denoise(a, self.bias_spec, strength, lengths=lengths)
        return out.squeeze(0) if squeeze else out
