"""mt_vconv's compile-time K loop (the decoder's convs and the upsamplers: VcSched in csrc/mt_vconv.hip) against the
runtime-cursor loop it replaces: same tiles, staging images and MFMA order, so the results must be BIT-identical.
Checked end to end through the bench's text->wav step (bf16 synthesize: every decoder conv of the U-Net,
model.py:964-1048, in both attention paths; the Generator's upsamplers, hifigan/models.py:183-185), at a small batch
(one-round grids) and at B = 40 (multi-round grids, odd / even tile counts per workgroup), plus the variants the
launches used (launch log)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _models():
    import bench
    return bench.build_models(DEV, "bf16", 1234)


def _run(models, x, xl, ct):
    import bench
    from matcha_hip import runtime as rt
    m, g, den, _, _ = models
    prev = rt.set_vconv_ct(ct)
    try:
        torch.manual_seed(7)  # the same CFM noise z for both runs (synthesize draws it with torch.randn_like)
        with torch.inference_mode():
            mel, yl, wav = bench.step(m, g, den, x, xl, 10, True)
        torch.cuda.synchronize()
    finally:
        rt.set_vconv_ct(prev)
    return mel.cpu(), yl.cpu(), wav.cpu()


@pytest.mark.parametrize("B,general", [(6, False), (40, False), (8, True)])
def test_compile_time_k_loop_bit_identical(B, general):
    import bench
    models = _models()
    x, xl = bench.shard_inputs(0, 1, B, 1234 + B)
    if general:  # the longest text a multiple of 4 tokens: y_max % 4 == 0, no padded frame -> general attention
        xl[0] = (int(xl.max()) // 4) * 4
        xl = torch.minimum(xl, xl[0])
        x = x[:, : int(xl[0])] * (torch.arange(int(xl[0]))[None] < xl[:, None])
    x, xl = x.to(DEV), xl.to(DEV)
    a = _run(models, x, xl, True)
    b = _run(models, x, xl, False)
    assert torch.equal(a[1], b[1])
    assert torch.equal(a[0], b[0])
    assert torch.equal(a[2], b[2])
    assert torch.isfinite(a[2]).all()


def test_compile_time_k_loop_variants_launched():
    """the bench step launches the compile-time variants it was built for: the decoder's GroupNorm / masked k = 3
    convs at C_in 192 / 256 / 512, the stride-2 down conv (2 taps over frame pairs, C_in 512), the LN-folded 1x1
    GEMMs, FF2 (C_in 1024, residual + mask), the residual GroupNorm 1x1 convs, the ConvTranspose up conv and the
    vocoder's upsamplers (plain outputs: the stage 1-2 conv1s activate their input themselves, VE_ACTIN; the launch
    log records (epilogue, C_in, taps))"""
    import bench
    from matcha_hip import runtime as rt
    m, g, den, _, _ = _models()
    x, xl = bench.shard_inputs(0, 1, 8, 1234)
    with torch.inference_mode():
        rt.vconv_log_start(20000)
        bench.step(m, g, den, x.to(DEV), xl.to(DEV), 10, True)
        torch.cuda.synchronize()
        recs = rt.vconv_log_stop(20000)
    seen = {(r["ef"], r["cin"] // 64, r["taps"]) for r in recs}
    GNSTATS, MASK, PMASK, DUAL = 256, 128, 4096, 16
    LNP_SNAKE, RESID_MASK, GNRES = 32 | 1024 | 64, 1 | 128, 1 | 512 | 8192
    for want in [(GNSTATS, 3, 3), (GNSTATS, 4, 3), (GNSTATS, 8, 3), (LNP_SNAKE, 4, 1), (RESID_MASK, 16, 1),
                 (GNRES, 4, 1), (MASK, 4, 3), (MASK, 8, 2), (PMASK, 4, 2), (0, 8, 2)]:
        assert want in seen, (want, sorted(seen))
