"""conv_post (hifigan/models.py:193-195: tanh(conv_post(leaky_relu(xs)))) folded into the last ResBlock pair of the
vocoder's final stage (mt_vpair32 VE_POST: the stage output xs never reaches HBM) against its own launch
(post_conv_kernel). Both run post_taps / post_combine's MFMA arithmetic (mt_vpair.h), so the waveforms must be EQUAL, on ragged and
padded batches, and the folded launch must really have run (launch log). Against the fp32 oracle the folded path is
what tests/test_gpu_parity_bf16.py and test_gpu_bench_shapes.py run (it is the default)."""
import pytest
import torch

from conftest import make_generator

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
VE_POST = 131072


def _gen(seed=31):
    from matcha_hip import synthetic
    gen = make_generator("bf16")
    sd = synthetic.make_state_dict([(k, tuple(v.shape)) for k, v in gen.state_dict().items()], seed)
    gen.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    gen = gen.to(DEV).eval()
    gen.remove_weight_norm()
    return gen


@pytest.mark.parametrize("ragged", [True, False])
def test_post_fold_bit_identical(ragged):
    from matcha_hip import runtime as rt
    gen = _gen()
    g = torch.Generator().manual_seed(4)
    B, T = 6, 230
    mel = (torch.randn(B, 80, T, generator=g) * 2.1 - 5.5).to(DEV)
    lens = torch.tensor([230, 181, 97, 230, 33, 150]).to(DEV) if ragged else None
    outs, posts = [], []
    for fold in (True, False):
        prev = rt.set_post_fold(fold)
        try:
            rt.vconv_log_start(20000)
            with torch.inference_mode():
                wav = gen(mel, lengths=lens) if ragged else gen(mel)
            torch.cuda.synchronize()
            log = rt.vconv_log_stop(20000)
        finally:
            rt.set_post_fold(prev)
        outs.append(wav.cpu())
        posts.append(sum(1 for r in log if r["ef"] & 0x10000 and r["ef"] & VE_POST))
    assert posts == [1, 0], posts
    assert torch.isfinite(outs[0]).all()
    assert torch.equal(outs[0], outs[1]), (outs[0] - outs[1]).abs().max().item()
    if ragged:  # samples past each utterance's 256 * length are zero (post_conv_kernel's and the fold's memset)
        for b, n in enumerate([230, 181, 97, 230, 33, 150]):
            assert float(outs[0][b, ..., 256 * n:].abs().max() if 256 * n < outs[0].shape[-1] else 0) == 0.0
