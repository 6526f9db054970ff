"""Op-level parity of the HIP kernels (implicit-GEMM conv, attention) on the MI355X.

References are plain PyTorch fp64 on CPU of the same op (floating-point kernels).
Tolerances: fp32 mode max-abs <= 2e-5 * sqrt(K) scale; bf16 mode rel-RMS <= 1e-2.
"""
import math

import pytest
import torch
import torch.nn.functional as F

from conftest import rel_rms

pytestmark = pytest.mark.gpu

CONV_CASES = [
    # cin, cout, k, stride, pad, dil, transposed, B, Tin, slope
    (80, 512, 7, 1, 3, 1, False, 2, 37, None),       # HiFi-GAN conv_pre (cin not a chunk multiple)
    (160, 256, 3, 1, 1, 1, False, 2, 64, None),      # U-Net first conv (C_cond 160)
    (224, 256, 1, 1, 0, 1, False, 1, 50, None),      # res_conv, VCTK C_cond
    (256, 256, 3, 2, 1, 1, False, 2, 64, None),      # Downsample1D k3 s2
    (256, 384, 1, 1, 0, 1, False, 3, 130, None),     # QKV projection
    (1024, 256, 1, 1, 0, 1, False, 1, 70, None),     # FF2
    (128, 128, 11, 1, 25, 5, False, 1, 300, 0.1),    # ResBlock1 k11 d5
    (64, 64, 7, 1, 9, 3, False, 2, 257, 0.1),        # ResBlock1 k7 d3
    (32, 32, 3, 1, 1, 1, False, 2, 1000, 0.1),       # last-stage resblock
    (32, 1, 7, 1, 3, 1, False, 2, 517, 0.01),        # conv_post (M = 1)
    (512, 256, 16, 8, 4, 1, True, 2, 17, 0.1),       # ups.0 polyphase ConvT k16 s8
    (128, 64, 4, 2, 1, 1, True, 1, 100, 0.1),        # ups.2 ConvT k4 s2
    (256, 256, 4, 2, 1, 1, True, 2, 32, None),       # U-Net Upsample1D
]


def _ref_conv(x_btc, W, b, stride, pad, dil, transposed, slope):
    x = x_btc.double().permute(0, 2, 1)
    if slope is not None:
        x = F.leaky_relu(x, slope)
    if transposed:
        y = F.conv_transpose1d(x, W.double(), b.double(), stride=stride, padding=pad)
    else:
        y = F.conv1d(x, W.double(), b.double(), stride=stride, padding=pad, dilation=dil)
    return y.permute(0, 2, 1)


@pytest.mark.parametrize("case", CONV_CASES, ids=lambda c: f"{c[0]}x{c[1]}k{c[2]}s{c[3]}d{c[5]}{'T' if c[6] else ''}")
@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_conv1d(case, precision):
    from matcha_hip import runtime as rt
    cin, cout, k, stride, pad, dil, tr, B, Tin, slope = case
    g = torch.Generator().manual_seed(cin * 7 + cout + k)
    x = torch.randn(B, Tin, cin, generator=g)
    fan = cin * k / (stride if tr else 1)
    W = torch.randn(*((cin, cout, k) if tr else (cout, cin, k)), generator=g) / math.sqrt(fan)
    b = 0.1 * torch.randn(cout, generator=g)
    if precision == "bf16":
        x = x.bfloat16().float()
    y = rt.op_conv1d(x.cuda(), W.cuda(), b.cuda(), stride, pad, dil, tr, slope, precision).float().cpu()
    if precision == "bf16":
        W = W.bfloat16().float()
    ref = _ref_conv(x, W, b, stride, pad, dil, tr, slope)
    assert y.shape == ref.shape
    if precision == "fp32":
        assert (y.double() - ref).abs().max() < 1e-5 * math.sqrt(cin * k) + 1e-6
    else:
        assert rel_rms(y, ref) < 1e-2


def _ref_attention(qkv, mask, heads):
    """model.py:686-701 semantics incl. the +3.4e38 masked-key fill, in fp64."""
    B, T, _ = qkv.shape
    inner = heads * 64
    q, k, v = qkv[..., :inner], qkv[..., inner:2 * inner], qkv[..., 2 * inner:]

    def sp(z):
        return z.double().view(B, T, heads, 64).permute(0, 2, 1, 3)

    q, k, v = sp(q), sp(k), sp(v)
    s = torch.einsum("bhid,bhjd->bhij", q, k) * 0.125
    m = mask.view(B, 1, 1, T)
    s = s.masked_fill(m == 0, -torch.finfo(torch.float32).min)
    p = s.softmax(-1)
    return torch.einsum("bhij,bhjd->bhid", p, v).permute(0, 2, 1, 3).reshape(B, T, inner)


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
@pytest.mark.parametrize("T,lens", [(64, [64, 53]), (300, [300, 300, 17]), (130, [129, 130])])
def test_attention_reference_mask_semantics(precision, T, lens):
    from matcha_hip import runtime as rt
    B, heads = len(lens), 2
    g = torch.Generator().manual_seed(T)
    qkv = torch.randn(B, T, 3 * heads * 64, generator=g) * 1.5
    mask = (torch.arange(T)[None] < torch.tensor(lens)[:, None]).float()
    if precision == "bf16":
        qkv = qkv.bfloat16().float()
    out = rt.op_attention(qkv.cuda(), mask.cuda(), heads, precision).float().cpu()
    ref = _ref_attention(qkv, mask, heads)
    for b in range(B):
        if precision == "fp32":
            assert (out[b].double() - ref[b]).abs().max() < 2e-5, b
        else:
            assert rel_rms(out[b], ref[b]) < 1e-2, b
    # padded utterances: every query gets the mean of the masked values (quirk), independent of q
    for b, L in enumerate(lens):
        if L < T:
            assert torch.allclose(out[b, 0], out[b, -1], atol=1e-6)


VCONV_CASES = [
    # cin, cout, k, dil, B, L, ef   (ef bits: 1 resid, 2 accumulate, 4 /div, 8 y=lrelu(v), 16 y2=lrelu(v))
    (128, 128, 11, 5, 2, 300, 1 | 16),     # stage-2 conv2 of a non-last pair: x + conv, and its lrelu copy
    (128, 128, 3, 1, 1, 1000, 8),          # stage-2 conv1: only lrelu(conv) is stored
    (256, 256, 7, 3, 2, 517, 1 | 2 | 4),   # stage-1 last pair of the last resblock: (xs + x + conv) / 3
    (128, 128, 7, 1, 3, 100, 1),           # shorter than one 256-frame tile, 3 utterances
    (256, 128, 3, 5, 2, 256, 1 | 2),       # exact tile multiple, accumulate
    (128, 256, 11, 1, 1, 40, 0),           # more padding than frames
    (64, 64, 11, 5, 2, 700, 1 | 16),       # 64-channel stage (64-row tiles)
    (64, 64, 3, 1, 3, 255, 1 | 2 | 4),     # 64-channel, accumulate + divide
]


@pytest.mark.parametrize("case", VCONV_CASES, ids=lambda c: f"{c[0]}x{c[1]}k{c[2]}d{c[3]}B{c[4]}L{c[5]}ef{c[6]}")
def test_vconv_lds_dma_conv(case):
    """mt_vconv (persistent LDS-DMA conv, bf16) against an fp64 CPU conv of the same bf16 operands:
    y = epilogue(conv1d(x, W, 'same' padding, dilation) + b). rel-RMS <= 4e-3 (bf16 output rounding)."""
    from matcha_hip import runtime as rt
    cin, cout, k, dil, B, L, ef = case
    g = torch.Generator().manual_seed(cin + 3 * cout + k * 11 + dil + B + L)
    x = torch.randn(B, L, cin, generator=g).bfloat16()
    W = (torch.randn(cout, cin, k, generator=g) / math.sqrt(cin * k)).bfloat16().float()
    b = 0.1 * torch.randn(cout, generator=g)
    resid = torch.randn(B, L, cout, generator=g).bfloat16()
    y0 = torch.randn(B, L, cout, generator=g).bfloat16()
    y = y0.cuda().clone()
    out, out2 = rt.op_vconv(x.cuda(), W.cuda(), b.cuda(), dil, ef, resid.cuda() if ef & 1 else None, y=y,
                            slope=0.1, div=3.0)
    torch.cuda.synchronize()
    v = F.conv1d(x.double().permute(0, 2, 1), W.double(), b.double(), padding=dil * (k - 1) // 2,
                 dilation=dil).permute(0, 2, 1)
    if ef & 1:
        v = v + resid.double()
    if ef & 2:
        v = y0.double() + v
    if ef & 4:
        v = v / 3.0
    ref = F.leaky_relu(v, 0.1) if ef & 8 else v
    assert rel_rms(out.double().cpu(), ref) <= 4e-3
    if ef & 16:
        assert rel_rms(out2.double().cpu(), F.leaky_relu(v, 0.1)) <= 4e-3
        # the activated copy is lrelu of the stored (rounded) value, exactly
        assert torch.equal(out2.cpu(), F.leaky_relu(out.float().cpu(), 0.1).bfloat16())
