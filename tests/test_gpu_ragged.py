"""Ragged vocoder + denoiser (each utterance of a padded batch at its own length; mt_ragged.h).

The reference vocodes and denoises one utterance per call, on the mel `synthesize` cropped to that utterance
(main.py:181-198, MOS_audiou_generator.ipynb:265-277). ``Generator.forward(mel, lengths)`` and
``Denoiser.forward(audio, strength, lengths)`` do it for a whole padded batch in one launch chain. Checked here:
  - every row equals the same engine's one-utterance call on the cropped mel / audio, BIT FOR BIT (the same tiles
    per utterance, the same MFMA accumulation order), and is zero past its length;
  - every row against the fp32 oracle's one-utterance call (rel-RMS 1e-2, the SURVEY §8c bf16 bar);
  - lengths 1 and 0 and a batch where every row is full (= the padded call);
  - the fp32 engine on the generic per-layer kernel (within fp32 accumulation order of its one-utterance calls).
"""
import pytest
import torch

from conftest import make_generator, rel_rms

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _gen(precision, seed=8):
    from matcha_hip import synthetic
    g = make_generator(precision)
    sd = synthetic.make_state_dict([(k, tuple(v.shape)) for k, v in g.state_dict().items()], seed)
    g.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    g = g.to(DEV).eval()
    g.remove_weight_norm()
    return g


def _mel(B, T, seed=9):
    return torch.randn(B, 80, T, generator=torch.Generator().manual_seed(seed)) * 2.1 - 5.5


@pytest.mark.parametrize("T", [16, 300])
def test_vocoder_rows_do_not_depend_on_the_batch(T):
    """A row's waveform is the same bits whatever else shares the launch: rows 0-7 vocoded alone, inside a batch of
    64 and inside one of 200, ragged and at full length (the generic conv kernel picked its tile configuration
    from the batch size, and its two configurations sum K in different orders: conv_pre's rows then moved with B;
    ConvArgs::fixed_tile)."""
    g = _gen("bf16")
    mel = _mel(200, T, seed=12).to(DEV)
    lens = torch.randint(1, T + 1, (200,), generator=torch.Generator().manual_seed(13)).to(DEV)
    for ln in (lens, None):
        ref = g(mel[:8].contiguous(), lengths=None if ln is None else ln[:8])
        for B in (64, 200):
            out = g(mel[:B].contiguous(), lengths=None if ln is None else ln[:B])
            assert torch.equal(out[:8], ref), (B, ln is None)


def test_vocoder_ragged_batch_beyond_one_launch_chain():
    """More utterances than one ragged launch chain takes (runtime.RAGGED_MAX_BATCH = 512, the kernels' LDS tile
    tables): Generator.forward vocodes consecutive chunks; every row equals the same row vocoded in a small ragged
    batch (bit for bit: rows are independent), and is zero past its length."""
    from matcha_hip import runtime as rt
    g = _gen("bf16")
    B, T = rt.RAGGED_MAX_BATCH + 5, 16
    lens = torch.randint(0, T + 1, (B,), generator=torch.Generator().manual_seed(3))
    lens[0], lens[-1] = T, 1
    mel = _mel(B, T, seed=4).to(DEV)
    wav = g(mel, lengths=lens.to(DEV))
    torch.cuda.synchronize()
    assert wav.shape == (B, 1, T * 256) and torch.isfinite(wav).all()
    for s in (0, rt.RAGGED_MAX_BATCH - 3):  # rows on both sides of the chunk boundary, re-vocoded as one small batch
        part = g(mel[s:s + 8].contiguous(), lengths=lens[s:s + 8].to(DEV))
        assert torch.equal(wav[s:s + 8], part), s
    for b in range(B):
        assert torch.count_nonzero(wav[b, :, int(lens[b]) * 256:]) == 0, b


def test_vocoder_ragged_rows_equal_one_utterance_calls():
    from hifigan.config import v1
    from matcha_hip import runtime as rt
    from oracle import matcha_oracle as O
    g = _gen("bf16")
    assert g.engine().ragged_supported()
    B, T = 7, 300
    lens = torch.tensor([300, 257, 129, 64, 299, 1, 0])
    mel = _mel(B, T).to(DEV)
    rt.vconv_log_start()
    wav = g(mel, lengths=lens.to(DEV))
    torch.cuda.synchronize()
    log = rt.vconv_log_stop()
    assert wav.shape == (B, 1, T * 256)
    # every ResBlock conv ran multi-tile on the ragged batch (stage 1: 2400 frames -> 10 tiles for the longest row)
    assert any(r["ntiles"] > r["grid"] for r in log if r["taps"] >= 3)
    gs = {k: v.cpu() for k, v in g.state_dict().items()}
    for b in range(B):
        n = int(lens[b])
        assert torch.count_nonzero(wav[b, :, n * 256:]) == 0, b
        if n == 0:
            continue
        one = g(mel[b:b + 1, :, :n].contiguous())
        assert torch.equal(wav[b:b + 1, :, :n * 256], one), (b, (wav[b, :, :n * 256] - one[0]).abs().max())
        if n >= 64:  # fp32 oracle on the cropped mel (the reference's one-utterance call)
            ref = O.generator_forward(gs, mel[b:b + 1, :, :n].cpu(), v1)
            err = rel_rms(wav[b:b + 1, :, :n * 256].cpu(), ref)
            print(f"row {b} n={n}: rel-RMS vs oracle {err:.3e}")
            assert err < 1e-2, (b, err)


def test_vocoder_ragged_full_rows_equal_padded_call():
    g = _gen("bf16")
    B, T = 3, 200
    mel = _mel(B, T, seed=3).to(DEV)
    full = g(mel)
    rag = g(mel, lengths=torch.full((B,), T, device=DEV))
    assert torch.equal(full, rag)


def test_vocoder_ragged_fp32_generic_kernel():
    """fp32 (parity mode): the generic per-layer kernel runs the ragged batch (ConvArgs::lens). Its tile shape may
    differ between the batch and a one-utterance call, so rows agree with the one-utterance calls to fp32
    accumulation order (1e-5, the fp32 waveform tolerance), and are zero past their lengths."""
    g = _gen("fp32")
    assert g.engine().ragged_supported()
    B, T = 3, 96
    lens = torch.tensor([96, 40, 17])
    mel = _mel(B, T, seed=5).to(DEV)
    wav = g(mel, lengths=lens.to(DEV))
    for b in range(B):
        n = int(lens[b])
        one = g(mel[b:b + 1, :, :n].contiguous())
        assert (wav[b:b + 1, :, :n * 256] - one).abs().max() < 1e-5, b
        assert torch.count_nonzero(wav[b, :, n * 256:]) == 0


def test_denoiser_ragged_rows_equal_one_utterance_calls():
    from hifigan.denoiser import Denoiser
    from oracle import matcha_oracle as O
    g = _gen("bf16")
    den = Denoiser(g, mode="zeros")
    B, T = 5, 60
    lens = torch.tensor([60, 33, 3, 59, 12])
    audio = (torch.randn(B, T * 256, generator=torch.Generator().manual_seed(4)) * 0.3).clamp(-1, 1).to(DEV)
    out = den(audio, strength=0.00025, lengths=lens.to(DEV))
    assert out.shape == (B, T * 256)
    bias = den.bias_spec.cpu()  # the oracle STFT / iSTFT on the same bias spectrum
    for b in range(B):
        n = int(lens[b]) * 256
        one = den(audio[b, :n].contiguous(), strength=0.00025)
        assert torch.equal(out[b, :n], one), (b, (out[b, :n] - one).abs().max())
        assert torch.count_nonzero(out[b, n:]) == 0
        ref = O.denoise(audio[b:b + 1, :n].cpu(), bias, 0.00025)[0]
        assert (out[b, :n].cpu() - ref).abs().max() < 1e-4, b
