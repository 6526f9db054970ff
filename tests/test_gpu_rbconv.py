"""mt_rbconv (the HiFi-GAN wide-stage ResBlock convs with a compile-time K-loop schedule, hifigan/models.py:90-97,
183-192) against the generic mt_vconv kernel it replaces: the same tiles, staging images and MFMA order, so every
output must be BIT-identical (y and the activated copy y2), for every epilogue the vocoder launches, C = 256 / 128,
k = 3 / 7 / 11 at dilations 1 / 3 / 5, ragged and padded batches, one-round, XCD-major and multi-round round-robin
grids, and odd / even tile counts per workgroup (the C = 128 kernel unrolls two tiles per body). The fp64 check of
the conv itself is tests/test_gpu_ops.py::test_vconv_lds_dma_conv, which now runs on mt_rbconv for these shapes."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)

ACT, RD, R, RA, RAD, RADD = 8, 1 | 16, 1, 1 | 2, 1 | 2 | 4, 1 | 2 | 4 | 16
ACTIN = 16384

# (C, k, dil, B, L, ef, ragged)
CASES = [
    (256, 3, 1, 2, 300, ACT, False),
    (256, 3, 3, 3, 517, RD, True),
    (256, 7, 5, 2, 700, ACT, True),
    (256, 7, 1, 2, 1000, RA, False),
    (256, 11, 5, 3, 640, RD, True),
    (256, 11, 1, 2, 513, RADD, True),
    (256, 3, 1, 1, 40, R, False),          # shorter than a tile
    (128, 7, 3, 3, 900, ACT, True),
    (128, 7, 1, 2, 770, RD, True),
    (128, 11, 5, 2, 1290, ACT, False),
    (128, 11, 1, 3, 1100, RADD, True),
    (128, 3, 5, 2, 600, RAD, False),
    (128, 7, 1, 1, 256, R, False),         # exactly one tile
    (256, 7, 3, 64, 600, RD, True),        # 384 tiles: XCD-major, 1-2 tiles per workgroup
    (256, 11, 5, 160, 600, ACT, True),     # > 3 rounds: the round-robin walk
    (128, 11, 1, 150, 1100, RADD, True),   # C = 128, > 3 rounds, odd and even tile counts per workgroup
    (128, 7, 5, 37, 1300, RD, False),
]


def _run(case, rb, extra_ef=0):
    from matcha_hip import runtime as rt
    C, k, dil, B, L, ef, ragged = case
    g = torch.Generator().manual_seed(C + 7 * k + 13 * dil + B + L + ef)
    ef |= extra_ef  # flags that must not change the inputs drawn
    x = torch.randn(B, L, C, generator=g).bfloat16()
    W = (torch.randn(C, C, k, generator=g) / math.sqrt(C * k)).float()
    b = 0.1 * torch.randn(C, generator=g)
    resid = torch.randn(B, L, C, generator=g).bfloat16()
    y0 = torch.randn(B, L, C, generator=g).bfloat16()
    lens = torch.randint(max(1, L // 3), L + 1, (B,), generator=g).int() if ragged else None
    if ragged:
        lens[0] = L
    prev = rt.set_rbconv(rb)
    try:
        y = y0.to(DEV).clone()
        y2 = torch.full((B, L, C), 7.0, dtype=torch.bfloat16, device=DEV) if ef & 16 else None
        out, out2 = rt.op_vconv(x.to(DEV), W.to(DEV), b.to(DEV), dil, ef, resid.to(DEV) if ef & 1 else None, y=y,
                                y2=y2, slope=0.1, div=3.0, lens=None if lens is None else lens.to(DEV))
        torch.cuda.synchronize()
    finally:
        rt.set_rbconv(prev)
    return out.cpu(), None if out2 is None else out2.cpu()


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"C{c[0]}k{c[1]}d{c[2]}B{c[3]}L{c[4]}ef{c[5]}{'r' if c[6] else ''}")
def test_rbconv_bit_identical_to_vconv(case):
    a, a2 = _run(case, True)
    b, b2 = _run(case, False)
    assert torch.equal(a, b)
    if a2 is not None:
        assert torch.equal(a2, b2)
    assert torch.isfinite(a.float()).all()


Y2ONLY = 32768


@pytest.mark.parametrize("C,k,dil,B,L,ragged", [(128, 11, 1, 3, 1100, True), (256, 11, 1, 2, 513, True),
                                                (128, 7, 1, 37, 1300, False)])
def test_rbconv_y2only_stores_the_same_y2_and_no_y(C, k, dil, B, L, ragged):
    """VE_Y2ONLY (the vocoder's stage-output conv2 when the next upsampler reads lrelu(xs) alone, mt_vconv.h):
    the activated copy is bit-identical to the VE_DUAL launch's and the raw y is not stored (it keeps the values
    the VE_ACCUM epilogue read), on the compile-time-schedule kernel whose per-tile store count changes; the generic
    kernel (mt_vconv) ignores the flag and stores y as before."""
    case = (C, k, dil, B, L, RADD, ragged)
    a, a2 = _run(case, True)
    c, c2 = _run(case, True, extra_ef=Y2ONLY)
    d, d2 = _run(case, False, extra_ef=Y2ONLY)
    assert torch.equal(a2, c2) and torch.equal(a2, d2)
    assert torch.equal(a, d)  # mt_vconv: y stored
    g = torch.Generator().manual_seed(C + 7 * k + 13 * dil + B + L + RADD)
    torch.randn(B, L, C, generator=g), torch.randn(C, C, k, generator=g), torch.randn(C, generator=g)
    torch.randn(B, L, C, generator=g)
    y0 = torch.randn(B, L, C, generator=g).bfloat16()
    assert torch.equal(c, y0)  # mt_rbconv: y untouched


def test_rbconv_runs_for_the_vocoder_convs():
    """the vocoder's stage 1-2 per-layer ResBlock convs are launched on mt_rbconv (launch log: the variant record is
    mt_vconv's, the dispatch is checked through the switch), and the bf16 Generator is bit-identical with it on / off
    on a ragged batch (every epilogue of the chain: ACT, RESID|DUAL, RESID, RESID|ACCUM, RESID|ACCUM|DIV|DUAL)"""
    from conftest import make_generator
    from matcha_hip import runtime as rt
    from matcha_hip import synthetic
    gen = make_generator("bf16")
    sd = synthetic.make_state_dict([(k, tuple(v.shape)) for k, v in gen.state_dict().items()], 31)
    gen.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    gen = gen.to(DEV).eval()
    gen.remove_weight_norm()
    g = torch.Generator().manual_seed(3)
    B, T = 6, 220
    mel = torch.randn(B, 80, T, generator=g).to(DEV)
    lens = torch.tensor([220, 180, 97, 220, 33, 150]).to(DEV)
    outs = []
    for rb in (True, False):
        prev = rt.set_rbconv(rb)
        try:
            with torch.inference_mode():
                outs.append(gen(mel, lengths=lens).cpu())
        finally:
            rt.set_rbconv(prev)
    assert torch.equal(outs[0], outs[1])


ACTIN_CASES = [(256, 3, 1, 2, 300, False), (256, 7, 5, 2, 700, True), (256, 11, 3, 3, 640, True), (128, 7, 3, 3, 900, True),
               (128, 11, 5, 2, 1290, False), (128, 3, 1, 1, 40, False), (128, 11, 1, 150, 1100, True),
               (256, 7, 1, 64, 600, True)]


@pytest.mark.parametrize("case", ACTIN_CASES, ids=lambda c: f"C{c[0]}k{c[1]}d{c[2]}B{c[3]}L{c[4]}{'r' if c[5] else ''}")
def test_rbconv_actin_equals_activated_input(case):
    """VE_ACTIN (conv1 reads the raw chain state and applies lrelu to its staged rows in LDS, one step before each
    chunk's first use) against VE_ACT on the activated copy the producers stored before, lrelu(bf16 x) rounded:
    bit-identical, over one-round, XCD-major and round-robin grids, ragged and padded"""
    from matcha_hip import runtime as rt
    C, k, dil, B, L, ragged = case
    g = torch.Generator().manual_seed(C + 3 * k + dil + B + L)
    x = torch.randn(B, L, C, generator=g).bfloat16()
    xa = torch.maximum(x.float(), 0.1 * x.float()).bfloat16()  # lrelu of the stored values (one rounding)
    W = (torch.randn(C, C, k, generator=g) / math.sqrt(C * k)).float()
    b = 0.1 * torch.randn(C, generator=g)
    lens = torch.randint(max(1, L // 3), L + 1, (B,), generator=g).int().to(DEV) if ragged else None
    outs = []
    for xin, ef in ((x, ACT | ACTIN), (xa, ACT)):
        y = torch.zeros(B, L, C, dtype=torch.bfloat16, device=DEV)
        out, _ = rt.op_vconv(xin.to(DEV), W.to(DEV), b.to(DEV), dil, ef, None, y=y, slope=0.1, lens=lens)
        torch.cuda.synchronize()
        outs.append(out.cpu())
    assert torch.equal(outs[0], outs[1])
    assert torch.isfinite(outs[0].float()).all()


def test_actin_vocoder_bit_identical():
    """the bf16 Generator with the stage 1-2 conv1s activating their input in LDS (no XA / RA copies stored) equals
    the one reading the producers' activated copies, on a ragged batch"""
    from conftest import make_generator
    from matcha_hip import runtime as rt
    from matcha_hip import synthetic
    gen = make_generator("bf16")
    sd = synthetic.make_state_dict([(k, tuple(v.shape)) for k, v in gen.state_dict().items()], 41)
    gen.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    gen = gen.to(DEV).eval()
    gen.remove_weight_norm()
    g = torch.Generator().manual_seed(5)
    B, T = 6, 220
    mel = torch.randn(B, 80, T, generator=g).to(DEV)
    lens = torch.tensor([220, 180, 97, 220, 33, 150]).to(DEV)
    outs = []
    for on in (True, False):
        prev = rt.set_rbconv_actin(on)
        try:
            with torch.inference_mode():
                outs.append(gen(mel, lengths=lens).cpu())
        finally:
            rt.set_rbconv_actin(prev)
    assert torch.equal(outs[0], outs[1])
