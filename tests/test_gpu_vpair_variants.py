"""Round-5 ResBlock pair kernels against the kernels they replace (mt_vpair_set_kernels): the compile-time K loops
(unrolled steps, constant ring slots and vmcnt counts, phantom prefetches past the last tile) of the 64-channel k = 7 /
11 pairs and the 128-channel k = 3 pairs (d = 1, 3, 5; fixed row staging spread over conv2's steps). Same fragments, MFMA accumulation order and rounding points, so the Generator's waveform must be BIT-identical
with the variant on and off (hifigan/models.py:90-97, 183-192), on a ragged batch (one-utterance tiles at each length)
and on a padded one, with multi-round grids (tile counts per workgroup of both parities: the k = 7 kernel's ring
slot base rotates per tile) and at batch 1 (one-round grids).
"""
import pytest
import torch

from conftest import make_generator

pytestmark = pytest.mark.gpu
DEV = "cuda"
VPK_ALL = 3  # mt_vpair.h: VPK_CTK | VPK_CTK128


def _gen(seed=8):
    from matcha_hip import synthetic
    g = make_generator("bf16")
    sd = synthetic.make_state_dict([(k, tuple(v.shape)) for k, v in g.state_dict().items()], seed)
    g.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    g = g.to(DEV).eval()
    g.remove_weight_norm()
    return g


def _run(g, mel, lens, mask):
    from matcha_hip import runtime as rt
    prev = rt.set_vpair_kernels(mask)
    try:
        with torch.inference_mode():
            wav = g(mel, lengths=lens) if lens is not None else g(mel)
        torch.cuda.synchronize()
    finally:
        rt.set_vpair_kernels(prev)
    return wav.cpu()


@pytest.mark.parametrize("B,T,ragged", [(7, 300, True), (24, 420, True), (5, 333, False), (1, 97, False)])
def test_round5_pair_kernels_bit_identical(B, T, ragged):
    g = _gen()
    mel = (torch.randn(B, 80, T, generator=torch.Generator().manual_seed(B + T)) * 2.1 - 5.5).to(DEV)
    lens = None
    if ragged:
        lens = torch.randint(T // 3, T + 1, (B,), generator=torch.Generator().manual_seed(T))
        lens[0] = T
        lens = lens.to(DEV)
    on = _run(g, mel, lens, VPK_ALL)
    assert torch.isfinite(on).all()
    off = _run(g, mel, lens, 0)
    assert torch.equal(on, off), (on - off).abs().max()
