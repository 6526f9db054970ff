"""Every library switch at the bench's own step (MI355X).

The library carries process-wide switches (mt_vconv_set_rbconv / _set_ct / _set_actin, mt_vpair_set_kernels,
mt_vocoder_set_post_fold, mt_ffn_set / _set_min_frames, mt_decoder_set_kernels) and per-engine ones (the decoder's
graphs / uniform attention / vconv mode, the vocoder's pair / vconv / fusion modes, the encoder's MFMA attention /
vconv). The parity tests check the DEFAULT path against the oracle; this module runs the exact bench step (bf16
text -> wav, B = 32, 10 Euler steps, denoiser; synthetic weights with the duration head forced, so every setting
sees the same y_lengths) once per non-default setting and compares it with the default run:

  * the switches that select a kernel variant computing the same operations in the same order must give the
    default's mel, y_lengths and waveform BIT FOR BIT (torch.equal);
  * the switches that change the arithmetic (another kernel family, the general attention instead of the
    query-independent one, the encoder's VALU attention or generic convs) must stay within the bf16 bar of the
    default on the mel (relative RMS 1e-2) and within 2e-2 on the denoised waveform: each bf16 run is
    within the 1e-2 bar of the fp32 oracle there (measured 9.6e-3 on this step, tests/test_gpu_bench_shapes.py), so
    two runs whose bf16 rounding points differ are up to about the sum apart (measured 1.02e-2 for a 6.7e-4 change
    of the mel); the measured differences are printed.

Every output must be finite (this test found NaN in conv_post's separate kernel: its last block read LDS rows it
never wrote through the MFMA's zero tap row, mt_vpair.h post_rot).

The env-only knobs (MT_XCD_TILES, MT_K1_TILES, MT_VPAIR3: read once per process) are not flipped here.
Reference: model.py:1264-1300 (synthesize), hifigan/models.py:181-197, hifigan/denoiser.py:62-68.
"""
import sys

import pytest
import torch

from conftest import REPO, rel_rms

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def bench_step():
    if REPO not in sys.path:
        sys.path.insert(0, REPO)
    import bench
    m, g, den, _, _ = bench.build_models(torch.device(DEV), "bf16", 1234)
    x, xl = bench.shard_inputs(0, 1, 32, 1234)
    x, xl = x.to(DEV), xl.to(DEV)

    def run():
        torch.manual_seed(7)  # the CFM noise (torch.randn_like on the device)
        mel, yl, wav = bench.step(m, g, den, x, xl, 10, True)
        torch.cuda.synchronize()
        return mel.clone(), yl.clone(), wav.clone()

    ref = run()
    assert all(torch.isfinite(t).all() for t in (ref[0], ref[2]))
    return m, g, run, ref


def _rt():
    from matcha_hip import runtime as rt
    return rt


def test_default_step_is_deterministic(bench_step):
    _, _, run, ref = bench_step
    out = run()
    assert all(torch.equal(a, b) for a, b in zip(out, ref))


# (name, apply() -> restore(), bit-identical?)
def _process_switches():
    rt = _rt()

    def flip(setter, value):
        def apply():
            prev = setter(value)
            return lambda: setter(prev)
        return apply

    return [
        ("rbconv off (mt_vconv for the stage 1-2 ResBlock convs)", flip(rt.set_rbconv, False), True),
        ("runtime-cursor vconv K loops", flip(rt.set_vconv_ct, False), True),
        ("round-4 pair kernels (vpair_set_kernels(0))", flip(rt.set_vpair_kernels, 0), True),
        ("conv_post unfolded", flip(rt.set_post_fold, 0), True),
        ("activated copies instead of VE_ACTIN", flip(rt.set_rbconv_actin, False), True),
        ("decoder FeedForward as two GEMMs", flip(rt.set_ffn, 0), True),
        ("mt_ffn schedule 1", flip(rt.set_ffn, 1), True),
        ("mt_ffn schedule 2 (FF1 epilogue overlapped)", flip(rt.set_ffn, 2), True),
        ("mt_ffn on every U-Net level", flip(rt.set_ffn_min_frames, 0), True),
        ("generic final projection + Euler update", flip(rt.set_decoder_kernels, 0), True),
    ]


def _engine_switches(m, g):
    dec = m.decoder.estimator.engine()
    enc = m.encoder.engine()
    voc = g.engine()

    def flip(setter, value, default):
        def apply():
            setter(value)
            return lambda: setter(default)
        return apply

    return [
        ("decoder without hipGraph replay", flip(dec.set_graphs, 0, 1), True),
        ("decoder GroupNorm as its own pass (set_vconv(2))", flip(dec.set_vconv, 2, 1), False),
        ("decoder generic conv kernel (set_vconv(0))", flip(dec.set_vconv, 0, 1), False),
        ("decoder general attention (no query-independent path)", flip(dec.set_uniform_attention, 0, 1), False),
        ("vocoder every 128-channel pair fused (set_pair(4))", flip(voc.set_pair, 4, 1), True),
        ("vocoder 128-channel stage per layer (set_pair(2))", flip(voc.set_pair, 2, 1), True),
        ("vocoder all ResBlocks per layer (set_pair(0))", flip(voc.set_pair, 0, 1), False),
        ("vocoder vconv for stages 1-2 only (set_vconv(1))", flip(voc.set_vconv, 1, 2), False),
        ("vocoder generic per-layer kernel (set_vconv(0))", flip(voc.set_vconv, 0, 2), False),
        ("vocoder without stage fusion (set_fusion(0))", flip(voc.set_fusion, 0, 1), False),
        ("encoder attention off MFMA", flip(enc.set_mfma_attention, 0, 1), False),
        ("encoder generic conv kernel", flip(enc.set_vconv, 0, 1), False),
    ]


def _check(run, ref, name, apply, bitwise):
    restore = apply()
    try:
        mel, yl, wav = run()
    finally:
        restore()
    assert torch.equal(yl, ref[1]), f"{name}: y_lengths changed"
    assert torch.isfinite(mel).all() and torch.isfinite(wav).all(), f"{name}: non-finite output"
    same = torch.equal(mel, ref[0]) and torch.equal(wav, ref[2])
    e_mel, e_wav = rel_rms(mel.float().cpu(), ref[0].float().cpu()), rel_rms(wav.float().cpu(), ref[2].float().cpu())
    print(f"{name}: {'bit-identical' if same else 'differs'} (mel rel-RMS {e_mel:.2e}, wav {e_wav:.2e})")
    if bitwise:
        assert same, f"{name}: not bit-identical (mel {e_mel:.2e}, wav {e_wav:.2e})"
    else:
        assert e_mel < 1e-2 and e_wav < 2e-2, (name, e_mel, e_wav)


@pytest.mark.parametrize("i", range(10))
def test_process_switch_at_bench_step(bench_step, i):
    _, _, run, ref = bench_step
    name, apply, bitwise = _process_switches()[i]
    _check(run, ref, name, apply, bitwise)


@pytest.mark.parametrize("i", range(12))
def test_engine_switch_at_bench_step(bench_step, i):
    m, g, run, ref = bench_step
    name, apply, bitwise = _engine_switches(m, g)[i]
    _check(run, ref, name, apply, bitwise)
    # the default is back: the next run equals the reference again
    out = run()
    assert all(torch.equal(a, b) for a, b in zip(out, ref)), f"{name}: default not restored"
