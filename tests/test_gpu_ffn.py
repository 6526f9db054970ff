"""mt_ffn (csrc/mt_ffn.hip): the decoder transformer block's FeedForward as one fused launch, against the two
mt_vconv launches it replaces (FF1 with the LayerNorm / SnakeBeta epilogue, FF2 with the residual [+ mask]
epilogue; model.py:580-609, 733-741): same accumulation order and epilogue operations, h rounded to bf16 where the
two-launch path stores it, so the results must be BIT-identical. Checked end to end through the bench's text->wav
step (bf16 synthesize: every transformer block of the U-Net at both levels, in both attention paths), at a small
batch (one tile per workgroup, partial last tile) and at B = 40 (several tiles per workgroup)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _models():
    import bench
    return bench.build_models(DEV, "bf16", 1234)


def _run(models, x, xl, mode):
    import bench
    from matcha_hip import runtime as rt
    m, g, den, _, _ = models
    prev = rt.set_ffn(mode)
    prev_min = rt.set_ffn_min_frames(0)  # every level, whatever its size
    try:
        torch.manual_seed(7)  # the same CFM noise z for both runs (synthesize draws it with torch.randn_like)
        with torch.inference_mode():
            mel, yl, wav = bench.step(m, g, den, x, xl, 10, True)
        torch.cuda.synchronize()
    finally:
        rt.set_ffn(prev)
        rt.set_ffn_min_frames(prev_min)
    return mel.cpu(), yl.cpu(), wav.cpu()


@pytest.mark.parametrize("B,general", [(6, False), (40, False), (8, True)])
def test_fused_feedforward_bit_identical(B, general):
    import bench
    models = _models()
    x, xl = bench.shard_inputs(0, 1, B, 4321 + B)
    if general:  # the longest text a multiple of 4 tokens: y_max % 4 == 0, no padded frame -> general attention
        xl[0] = (int(xl.max()) // 4) * 4
        xl = torch.minimum(xl, xl[0])
        x = x[:, : int(xl[0])] * (torch.arange(int(xl[0]))[None] < xl[:, None])
    x, xl = x.to(DEV), xl.to(DEV)
    b = _run(models, x, xl, 0)
    for mode in (1, 2, 3):  # the serial schedule, the overlapped FF1 epilogues, frame-only prefetch
        a = _run(models, x, xl, mode)
        assert torch.equal(a[1], b[1])
        assert torch.equal(a[0], b[0]), (mode, (a[0] - b[0]).abs().max())
        assert torch.equal(a[2], b[2])
        assert torch.isfinite(a[0]).all()


def test_fused_feedforward_replaces_the_gemm_pair():
    """with mt_ffn on, the step's launch log holds no FF1 (VE_LN | VE_LNP | VE_SNAKE) or FF2 (C_in 1024) mt_vconv
    launch; with it off, 6 blocks x 10 steps of each"""
    import bench
    from matcha_hip import runtime as rt
    m, g, den, _, _ = _models()
    x, xl = bench.shard_inputs(0, 1, 8, 1234)
    FF1 = 32 | 1024 | 64
    counts = {}
    for fused in (True, False):
        prev = rt.set_ffn(fused)
        prev_min = rt.set_ffn_min_frames(0)
        try:
            with torch.inference_mode():
                rt.vconv_log_start(20000)
                bench.step(m, g, den, x.to(DEV), xl.to(DEV), 10, True)
                torch.cuda.synchronize()
                recs = rt.vconv_log_stop(20000)
        finally:
            rt.set_ffn(prev)
            rt.set_ffn_min_frames(prev_min)
        counts[fused] = (sum(1 for r in recs if r["ef"] == FF1), sum(1 for r in recs if r["cin"] == 1024))
    assert counts[True] == (0, 0), counts
    assert counts[False] == (60, 60), counts
