"""§8f rank 3, the CFM training step on the GPU (matcha_hip.train) against torch autograd through the oracle
(oracle/matcha_oracle.py: training_losses restates train_standalone.py:623-667 in plain torch, so autograd
on it is the gradient oracle). Per-primitive forward/backward checks first (conv / transposed conv via
im2col + exact-fp32 MFMA GEMM, GroupNorm, LayerNorm, SnakeBeta, masked softmax in both reference mask modes,
RoPE, embedding, dropout, Adam + clip), then the whole step: losses, the MAS path, every parameter's
gradient and the Adam update. fp32 throughout; tolerances are stated per test."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import HP, make_matcha, rel_rms
from matcha_hip import synthetic

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _tr():
    from matcha_hip import train
    return train


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


# ----------------------------------------------------------------------------------------- primitives
@pytest.mark.parametrize("ta,tb,M,N,K,batch", [(0, 0, 70, 33, 19, 1), (1, 0, 64, 64, 100, 3), (0, 1, 5, 130, 64, 2),
                                               (1, 1, 17, 9, 3, 1), (0, 0, 300, 260, 132, 2),
                                               (1, 0, 40, 70, 5000, 1), (0, 1, 200, 96, 3001, 1)])
def test_gemm_f32(ta, tb, M, N, K, batch):
    """vector (aligned leading dimensions) and scalar loads, partial tiles, batch strides, the bias / row-mask
    epilogue, and the split-K path (the last two cases: few tiles, long K, per-slice partials summed in order,
    epilogue in the reduction)"""
    tr = _tr()
    g = torch.Generator().manual_seed(M * N + K)
    A = torch.randn(batch, *((K, M) if ta else (M, K)), generator=g)
    B = torch.randn(batch, *((N, K) if tb else (K, N)), generator=g)
    C0 = torch.randn(batch, M, N, generator=g)
    bias = torch.randn(N, generator=g)
    rmask = (torch.rand(batch, M, generator=g) > 0.3).float()
    out = C0.clone().to(DEV)
    bias_d, rmask_d = bias.to(DEV), rmask.to(DEV)
    tr.gemm(A.to(DEV), B.to(DEV), M, N, K, out, ta=ta, tb=tb, alpha=0.5, beta=-1.0, batch=batch,
            sA=A[0].numel(), sB=B[0].numel(), sC=M * N, bias=bias_d, rmask=rmask_d)
    Ad = A.double().transpose(1, 2) if ta else A.double()
    Bd = B.double().transpose(1, 2) if tb else B.double()
    ref = (0.5 * Ad @ Bd - C0.double() + bias.double()) * rmask.double()[:, :, None]
    assert _rel(out, ref) < 2e-6


@pytest.mark.parametrize("fmt,dt", [(1, torch.float16), (2, torch.bfloat16)])
@pytest.mark.parametrize("ta,tb,M,N,K,batch", [(0, 0, 70, 33, 19, 1), (1, 0, 64, 64, 100, 3), (0, 1, 5, 130, 64, 2),
                                               (1, 1, 17, 9, 3, 1), (0, 0, 300, 260, 132, 2),
                                               (1, 0, 40, 70, 5000, 1), (0, 1, 200, 96, 3001, 1)])
def test_gemm_16bit_operands(fmt, dt, ta, tb, M, N, K, batch):
    """the mixed-precision GEMM ("16-mixed" fp16 / "bf16-mixed" bf16 operands, fp32 sums and fp32 output): equal,
    up to fp32 summation order, to the fp64 product of the RNE-rounded operands (autocast's matmul arithmetic
    without its 16-bit output rounding), on the same shapes, epilogue and split-K cases as the fp32 GEMM"""
    tr = _tr()
    g = torch.Generator().manual_seed(M * N + K + fmt)
    A = torch.randn(batch, *((K, M) if ta else (M, K)), generator=g) * 3.0
    B = torch.randn(batch, *((N, K) if tb else (K, N)), generator=g)
    C0 = torch.randn(batch, M, N, generator=g)
    bias = torch.randn(N, generator=g)
    rmask = (torch.rand(batch, M, generator=g) > 0.3).float()
    out = C0.clone().to(DEV)
    tr.gemm(A.to(DEV), B.to(DEV), M, N, K, out, ta=ta, tb=tb, alpha=0.5, beta=-1.0, batch=batch,
            sA=A[0].numel(), sB=B[0].numel(), sC=M * N, bias=bias.to(DEV), rmask=rmask.to(DEV), fmt=fmt)
    Ar, Br = A.to(dt).double(), B.to(dt).double()
    Ad = Ar.transpose(1, 2) if ta else Ar
    Bd = Br.transpose(1, 2) if tb else Br
    ref = (0.5 * Ad @ Bd - C0.double() + bias.double()) * rmask.double()[:, :, None]
    assert _rel(out, ref) < 2e-6
    # and it is not the fp32 product: the operand rounding is visible
    exact = (0.5 * (A.double().transpose(1, 2) if ta else A.double()) @ (B.double().transpose(1, 2) if tb
             else B.double()) - C0.double() + bias.double()) * rmask.double()[:, :, None]
    assert _rel(out, exact) > 1e-5


@pytest.mark.parametrize("k,stride,pad,dil", [(3, 1, 1, 1), (3, 2, 1, 1), (5, 1, 2, 1), (3, 1, 2, 2), (1, 1, 0, 1)])
def test_conv_fwd_bwd(k, stride, pad, dil):
    tr = _tr()
    g = torch.Generator().manual_seed(k * 10 + stride)
    B, T, Cin, Cout = 2, 37, 24, 40
    x = torch.randn(B, T, Cin, generator=g, requires_grad=True)
    W = torch.randn(Cout, Cin, k, generator=g, requires_grad=True)
    b = torch.randn(Cout, generator=g, requires_grad=True)
    y = F.conv1d(x.transpose(1, 2), W, b, stride=stride, padding=pad, dilation=dil).transpose(1, 2)
    dy = torch.randn(y.shape, generator=g)
    gx, gW, gb = torch.autograd.grad(y, (x, W, b), dy)
    yd, ctx = tr.conv_fwd(x.detach().to(DEV).contiguous(), W.detach().to(DEV), b.detach().to(DEV), stride, pad, dil)
    gWd, gbd = torch.empty_like(W, device=DEV), torch.empty_like(b, device=DEV)
    gxd = tr.conv_bwd(dy.to(DEV).contiguous(), ctx, W.detach().to(DEV), gWd, gbd)
    assert _rel(yd, y) < 1e-6 and _rel(gxd, gx) < 1e-6 and _rel(gWd, gW) < 1e-6 and _rel(gbd, gb) < 1e-6


def test_conv_transpose_fwd_bwd():
    tr = _tr()
    g = torch.Generator().manual_seed(5)
    B, Tin, Cin, Cout = 2, 19, 32, 24
    x = torch.randn(B, Tin, Cin, generator=g, requires_grad=True)
    W = torch.randn(Cin, Cout, 4, generator=g, requires_grad=True)
    b = torch.randn(Cout, generator=g, requires_grad=True)
    y = F.conv_transpose1d(x.transpose(1, 2), W, b, stride=2, padding=1).transpose(1, 2)
    dy = torch.randn(y.shape, generator=g)
    gx, gW, gb = torch.autograd.grad(y, (x, W, b), dy)
    yd, ctx = tr.convT_fwd(x.detach().to(DEV).contiguous(), W.detach().to(DEV), b.detach().to(DEV), 2, 1)
    gWd, gbd = torch.empty_like(W, device=DEV), torch.empty_like(b, device=DEV)
    gxd = tr.convT_bwd(dy.to(DEV).contiguous(), ctx, W.detach().to(DEV), gWd, gbd)
    assert yd.shape == y.shape
    assert _rel(yd, y) < 1e-6 and _rel(gxd, gx) < 1e-6 and _rel(gWd, gW) < 1e-6 and _rel(gbd, gb) < 1e-6


def test_groupnorm_layernorm_fwd_bwd():
    tr = _tr()
    g = torch.Generator().manual_seed(6)
    B, T, C = 3, 29, 64
    x = (torch.randn(B, T, C, generator=g) * 3 + 1).requires_grad_(True)
    gam = torch.randn(C, generator=g, requires_grad=True)
    bet = torch.randn(C, generator=g, requires_grad=True)
    dy = torch.randn(B, T, C, generator=g)
    y = F.group_norm(x.transpose(1, 2), 8, gam, bet, eps=1e-5).transpose(1, 2)
    ref = torch.autograd.grad(y, (x, gam, bet), dy)
    yd, ctx = tr.gn_fwd(x.detach().to(DEV).contiguous(), gam.detach().to(DEV), bet.detach().to(DEV))
    gg, gb = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
    dx = tr.gn_bwd(dy.to(DEV).contiguous(), ctx, gam.detach().to(DEV), gg, gb)
    assert _rel(yd, y) < 1e-6
    for a, b in zip((dx, gg, gb), ref):
        assert _rel(a, b) < 1e-5
    for eps in (1e-5, 1e-4):
        y = F.layer_norm(x, (C,), gam, bet, eps=eps)
        ref = torch.autograd.grad(y, (x, gam, bet), dy)
        yd, ctx = tr.ln_fwd(x.detach().to(DEV).contiguous(), gam.detach().to(DEV), bet.detach().to(DEV), eps)
        dx = tr.ln_bwd(dy.to(DEV).contiguous(), ctx, gam.detach().to(DEV), gg, gb)
        assert _rel(yd, y) < 1e-6
        for a, b in zip((dx, gg, gb), ref):
            assert _rel(a, b) < 1e-5


def test_snake_mish_silu_relu_bwd():
    tr = _tr()
    g = torch.Generator().manual_seed(7)
    x = (torch.randn(50, 96, generator=g) * 2).requires_grad_(True)
    la = (torch.randn(96, generator=g) * 0.3).requires_grad_(True)
    lb = (torch.randn(96, generator=g) * 0.3).requires_grad_(True)
    dy = torch.randn(50, 96, generator=g)
    y = x + 1.0 / (torch.exp(lb) + 1e-9) * torch.sin(x * torch.exp(la)) ** 2  # model.py:600-609
    ref = torch.autograd.grad(y, (x, la, lb), dy)
    xd = x.detach().to(DEV).contiguous()
    dx, ga, gb = torch.empty_like(xd), torch.empty_like(xd), torch.empty_like(xd)
    yd = torch.empty_like(xd)
    L = tr.lib()
    la_d, lb_d, dy_d = la.detach().to(DEV), lb.detach().to(DEV), dy.to(DEV)  # kept alive across the calls
    tr.check(L.mtt_snake_fwd(xd.data_ptr(), la_d.data_ptr(), lb_d.data_ptr(), xd.numel(), 96, yd.data_ptr(),
                             tr._s(xd)))
    tr.check(L.mtt_snake_bwd(xd.data_ptr(), la_d.data_ptr(), lb_d.data_ptr(), dy_d.data_ptr(), xd.numel(), 96,
                             dx.data_ptr(), ga.data_ptr(), gb.data_ptr(), tr._s(xd)))
    assert _rel(yd, y) < 1e-6 and _rel(dx, ref[0]) < 1e-5
    assert _rel(ga.sum(0), ref[1]) < 1e-5 and _rel(gb.sum(0), ref[2]) < 1e-5
    for op, opb, fn in ((tr.MISH, tr.MISH_B, lambda v: v * torch.tanh(F.softplus(v))), (tr.SILU, tr.SILU_B, F.silu),
                        (tr.RELU, tr.RELU_B, torch.relu)):
        y = fn(x)
        (gx,) = torch.autograd.grad(y, (x,), dy)
        assert _rel(tr.act(op, xd), y) < 1e-6
        assert _rel(tr.act_bwd(opb, xd, dy.to(DEV).contiguous()), gx) < 1e-5


@pytest.mark.parametrize("mode", [0, 1])
def test_masked_attention_fwd_bwd(mode):
    """mode 0: decoder key mask filled with -finfo.min = +3.4e38 (model.py:697, padded queries and keys attend
    uniformly to the padded keys); mode 1: encoder query x key mask filled with -1e4 (model.py:360) plus dropout
    off. Reference math in fp64 autograd."""
    tr = _tr()
    g = torch.Generator().manual_seed(8 + mode)
    B, T, H, dh = 3, 21, 2, 16
    lens = torch.tensor([21, 15, 8])
    m = (torch.arange(T)[None] < lens[:, None]).float()
    q, k, v = (torch.randn(B, T, H * dh, generator=g, dtype=torch.float64, requires_grad=True) for _ in range(3))
    scale = dh ** -0.5

    def heads(z):
        return z.view(B, T, H, dh).permute(0, 2, 1, 3)

    s = torch.einsum("bhid,bhjd->bhij", heads(q), heads(k)) * scale
    if mode == 0:
        s = s.masked_fill(m[:, None, None, :] == 0, 3.4028234663852886e38)
    else:
        s = s.masked_fill((m[:, None, :, None] * m[:, None, None, :]) == 0, -1e4)
    o = torch.einsum("bhij,bhjd->bhid", s.softmax(-1), heads(v)).permute(0, 2, 1, 3).reshape(B, T, H * dh)
    do = torch.randn(o.shape, generator=g, dtype=torch.float64)
    ref = torch.autograd.grad(o, (q, k, v), do)
    md = m.to(DEV)
    od, ctx = tr.attention_fwd(*(z.detach().float().to(DEV).contiguous() for z in (q, k, v)), md,
                               md if mode == 1 else None, H, dh, scale, mode)
    grads = tr.attention_bwd(do.float().to(DEV).contiguous(), ctx)
    assert _rel(od, o) < 1e-5
    for a, b in zip(grads, ref):
        assert _rel(a, b) < 1e-4


def test_rope_and_inverse():
    import oracle.matcha_oracle as O
    tr = _tr()
    from matcha_hip import runtime as rt
    g = torch.Generator().manual_seed(9)
    B, T, H, dh = 2, 13, 2, 96
    x = torch.randn(B, T, H * dh, generator=g)
    d = int(dh * 0.5)
    ref = O.rope(x.view(B, T, H, dh).permute(0, 2, 1, 3), d).permute(0, 2, 1, 3).reshape(B, T, H * dh)
    xd = x.to(DEV).contiguous()
    theta = rt.rope_theta(dh).to(DEV)
    tr.rope_(xd, H, dh, d, theta)
    assert _rel(xd, ref) < 1e-6
    tr.rope_(xd, H, dh, d, theta, inverse=True)
    assert _rel(xd, x) < 1e-6


def test_embedding_dropout_sums():
    tr = _tr()
    g = torch.Generator().manual_seed(10)
    V, C, B, T = 50, 24, 3, 17
    ids = torch.randint(0, V, (B, T), generator=g)
    dout = torch.randn(B * T, C, generator=g)
    table = torch.randn(V, C, generator=g)
    want = torch.zeros(V, C).index_add_(0, ids.view(-1), dout) * math.sqrt(C)
    got = torch.empty(V, C, device=DEV)
    ids_d, dout_d, table_d = ids.to(DEV), dout.to(DEV), table.to(DEV)
    tr.check(tr.lib().mtt_embed_bwd(ids_d.data_ptr(), B * T, dout_d.data_ptr(), V, C, math.sqrt(C), got.data_ptr(),
                                    tr._s(got)))
    assert _rel(got, want) < 1e-6
    out = torch.empty(B * T, C, device=DEV)
    tr.check(tr.lib().mtt_embed_fwd(ids_d.data_ptr(), B * T, table_d.data_ptr(), C, math.sqrt(C), out.data_ptr(),
                                    tr._s(out)))
    assert torch.equal(out.cpu(), table[ids.view(-1)] * math.sqrt(C))
    # dropout: keep rate, scaling, same mask for the same seed, different mask for another seed
    x = torch.ones(1 << 20, device=DEV)
    a, b, c = tr.dropout(x, 0.3, 77), tr.dropout(x, 0.3, 77), tr.dropout(x, 0.3, 78)
    assert torch.equal(a, b) and not torch.equal(a, c)
    keep = (a != 0).float().mean().item()
    assert abs(keep - 0.7) < 3e-3
    assert torch.allclose(a[a != 0], torch.full_like(a[a != 0], 1 / 0.7))
    # colsum (segmented) and full sum
    y = torch.randn(300, 70, generator=g)
    cs = tr.colsum(y.to(DEV), 70, torch.empty(3, 70, device=DEV), seg=100)
    assert _rel(cs, y.view(3, 100, 70).sum(1)) < 1e-6
    assert abs(tr.total(y.to(DEV)).item() - y.double().sum().item()) < 1e-3


def test_adam_and_clip_match_torch():
    """mtt_clip_factor + mtt_adam against torch.nn.utils.clip_grad_norm_(5.0) + torch.optim.Adam(lr) over 3 steps,
    both the clipping (large gradients) and non-clipping regimes, and the world-2 averaging fold."""
    tr = _tr()
    g = torch.Generator().manual_seed(11)
    n = 5000
    p0 = torch.randn(n, generator=g)
    for world, gscale in ((1, 0.01), (1, 1.0), (2, 1.0)):
        p_ref = p0.clone().requires_grad_(True)
        opt = torch.optim.Adam([p_ref], lr=1e-3)
        p, m, v = p0.to(DEV), torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
        for step in range(1, 4):
            gr = torch.randn(n, generator=g) * gscale
            p_ref.grad = gr.clone()
            torch.nn.utils.clip_grad_norm_([p_ref], 5.0)
            opt.step()
            gsum = (gr * world).to(DEV)  # the flat buffer after a SUM all-reduce of identical rank gradients
            sc, sumsq = torch.empty(2, device=DEV), tr.total(gsum, gsum)
            tr.check(tr.lib().mtt_clip_factor(sumsq.data_ptr(), 5.0, 1.0 / world, sc.data_ptr(), sc[1:].data_ptr(),
                                              tr._s(sc)))
            tr.check(tr.lib().mtt_adam(p.data_ptr(), gsum.data_ptr(), m.data_ptr(), v.data_ptr(), n, sc.data_ptr(),
                                       1e-3, 0.9, 0.999, 1e-8, step, tr._s(p)))
            assert abs(sc[1].item() - gr.norm().item()) / gr.norm().item() < 1e-5
        assert (p.cpu() - p_ref.detach()).abs().max().item() < 1e-6


# ----------------------------------------------------------------------------------------- the step
def _setup(seed=21, B=3, Tx=17, Ty=64, x_len=(17, 12, 9), y_len=(64, 50, 33)):
    m = make_matcha(1, "fp32")
    sd = {k: torch.from_numpy(v) for k, v in synthetic.make_state_dict(
        [(k, tuple(v.shape)) for k, v in m.state_dict().items()], seed).items()}
    g = torch.Generator().manual_seed(seed)
    xl, yl = torch.tensor(x_len), torch.tensor(y_len)
    x = torch.randint(1, 178, (B, Tx), generator=g) * (torch.arange(Tx)[None] < xl[:, None])
    y = torch.randn(B, 80, Ty, generator=g) * 1.5 * (torch.arange(Ty)[None, None] < yl[:, None, None])
    t = torch.rand(B, generator=g)
    z = torch.randn(B, 80, Ty, generator=g)
    return sd, x, xl, y, yl, t, z


def _configs4_batch(seed=41, B=64, Tx=200, Ty=868):
    """configs[4]'s batch: 64 LJSpeech-shaped utterances (train_standalone.py's batch_size 64), text 80..200
    tokens, mel ≈ 4.3 frames per token, the longest at T_y = 868 (T_y % 4 == 0, no fix_len padding needed)."""
    rs = np.random.RandomState(seed)
    x_len = rs.randint(80, Tx + 1, B)
    x_len[0] = Tx
    y_len = np.minimum(Ty, np.round(x_len * rs.uniform(3.6, 4.34, B))).astype(int)
    y_len[0] = Ty
    return _setup(seed=seed, B=B, Tx=Tx, Ty=Ty, x_len=tuple(int(v) for v in x_len),
                  y_len=tuple(int(v) for v in y_len))


def _oracle_grads(sd, x, xl, y, yl, t, z, mas=None):
    import oracle.matcha_oracle as O
    params = {k: v.clone().float().requires_grad_(True) for k, v in sd.items()
              if k.startswith(("encoder.", "decoder.estimator."))}
    dur, prior, cfm, attn, lp = O.training_losses(params, x, xl, y, yl, t, z, HP, mas=mas)
    grads = torch.autograd.grad(dur + prior + cfm, list(params.values()), allow_unused=True)
    return (dur, prior, cfm, attn, lp), {k: (gr if gr is not None else torch.zeros_like(p))
                                         for (k, p), gr in zip(params.items(), grads)}


def test_training_step_matches_autograd():
    """Losses (rel 1e-4), the MAS path (exact), the log-prior (rel 1e-5) and every parameter gradient (relative
    L2 error < 2e-3 per tensor, < 5e-4 over the whole flat gradient) of the fp32 GPU step against fp32 torch
    autograd through the oracle on the CPU (the reference's arithmetic order for the time embedding and the
    log-prior) on the same weights, batch, t and z (dropout off: eval-mode modules)."""
    _check_step(*_setup())


def test_training_step_configs4_size_matches_autograd():
    """The same checks at configs[4]'s per-GPU size: B = 64, T_x = 200, T_y = 868 (55.5 k mel frames), where the
    long-K weight gradients take the split-K GEMM path and every GEMM runs multi-tile. The oracle runs on the
    host CPU (the MAS in its anti-diagonal form, equal to the loop form: tests/test_mas.py)."""
    import oracle.matcha_oracle as O
    _check_step(*_configs4_batch(), mas=O.maximum_path_diag)


def test_training_configs4_size_dropout_deterministic():
    """Dropout on at configs[4]'s size: two trainers from the same weights and seed give bit-identical losses and
    gradients (fixed-order reductions, split-K included), and the masks change the loss against eval mode."""
    from matcha_hip.train import MatchaTrainer
    sd, x, xl, y, yl, t, z = _configs4_batch(seed=42)
    args = (x.to(DEV), xl.to(DEV), y.to(DEV), yl.to(DEV))
    kw = dict(t=t.to(DEV), z=z.to(DEV))
    outs, grads = [], []
    for _ in range(2):
        tr = MatchaTrainer(sd, HP, DEV, seed=9)
        outs.append(tr.forward_backward(*args, **kw)["loss"].item())
        grads.append(tr.grads.flat.detach().cpu().clone())
        del tr
    ev = MatchaTrainer(sd, HP, DEV, dropout=False).forward_backward(*args, **kw)["loss"].item()
    assert outs[0] == outs[1] and torch.equal(grads[0], grads[1])
    assert math.isfinite(outs[0]) and outs[0] != ev


def _check_step(sd, x, xl, y, yl, t, z, mas=None):
    from matcha_hip.train import MatchaTrainer
    (dur, prior, cfm, attn, lp), gref = _oracle_grads(sd, x, xl, y, yl, t, z, mas=mas)
    tr = MatchaTrainer(sd, HP, DEV, dropout=False)
    out = tr.forward_backward(x.to(DEV), xl.to(DEV), y.to(DEV), yl.to(DEV), t=t.to(DEV), z=z.to(DEV))
    torch.cuda.synchronize()
    assert torch.equal(out["attn"].cpu(), attn.float())
    assert _rel(out["log_prior"], lp) < 1e-5
    for name, a, b in (("dur", out["dur_loss"], dur), ("prior", out["prior_loss"], prior), ("cfm", out["cfm_loss"], cfm)):
        assert abs(a.item() - b.item()) <= 1e-4 * abs(b.item()), (name, a.item(), b.item())
    got = tr.gradients()
    # the encoder's key bias adds q.b to every score of a row: softmax is invariant to it, so its true gradient
    # is 0 and both sides hold rounding noise; it is checked against the scale of the key weight's gradient
    kb = [k for k in gref if k.endswith("conv_k.bias")]
    for k in kb:
        assert float((got[k].cpu() - gref[k]).norm()) <= 1e-3 * float(gref[k[:-4] + "weight"].norm()), k
    worst = max((_rel(got[k], gref[k]), k) for k in gref if k not in kb)
    assert worst[0] < 2e-3, worst
    flat_ref = torch.cat([gref[n].reshape(-1) for n in tr.grads.names])
    assert _rel(tr.grads.flat, flat_ref) < 5e-4
    # the duration loss trains proj_w only (its input is detached, model.py:532)
    assert all(gref[k].norm() > 0 for k in gref if k.startswith("encoder.proj_w."))


def test_training_step_adam_update_matches_torch():
    """optimizer_step on the GPU gradients vs clip_grad_norm_(5.0) + Adam(lr 1e-4) applied by torch to the SAME
    gradients: the update is isolated from gradient rounding (max |dp| error 5e-7, a few ulp of the weights)."""
    from matcha_hip.train import MatchaTrainer
    sd, x, xl, y, yl, t, z = _setup(seed=22)
    tr = MatchaTrainer(sd, HP, DEV, dropout=False)
    tr.forward_backward(x.to(DEV), xl.to(DEV), y.to(DEV), yl.to(DEV), t=t.to(DEV), z=z.to(DEV))
    g = {k: v.detach().cpu().clone() for k, v in tr.gradients().items()}
    p0 = {k: v.detach().cpu().clone() for k, v in tr.parameters().items()}
    tr.optimizer_step()
    ref = {k: p0[k].clone().requires_grad_(True) for k in tr.grads.names}
    for k, p in ref.items():
        p.grad = g[k].clone()
    norm = torch.nn.utils.clip_grad_norm_(list(ref.values()), 5.0)
    torch.optim.Adam(list(ref.values()), lr=1e-4).step()
    assert abs(tr.last["grad_norm"].item() - norm.item()) <= 1e-5 * norm.item()
    err = max(float((tr.parameters()[k].cpu() - ref[k].detach()).abs().max()) for k in ref)
    assert err < 5e-7


def test_training_with_dropout_is_deterministic_and_learns():
    """Dropout on (p = 0.1 encoder, 0.5 prenet, 0.1 duration predictor, 0.05 estimator): two trainers from the
    same weights and seed produce bit-identical losses and parameters (no atomics anywhere), the dropout
    masks change the loss against the eval-mode step, and 12 Adam steps on one batch lower the loss."""
    from matcha_hip.train import MatchaTrainer
    sd, x, xl, y, yl, t, z = _setup(seed=23)
    args = (x.to(DEV), xl.to(DEV), y.to(DEV), yl.to(DEV))
    a, b = MatchaTrainer(sd, HP, DEV, seed=5), MatchaTrainer(sd, HP, DEV, seed=5)
    ev = MatchaTrainer(sd, HP, DEV, dropout=False).forward_backward(*args, t=t.to(DEV), z=z.to(DEV))["loss"].item()
    losses = []
    for step in range(12):
        la = a.forward_backward(*args, t=t.to(DEV), z=z.to(DEV))["loss"].item()
        a.optimizer_step()
        if step < 2:
            lb = b.forward_backward(*args, t=t.to(DEV), z=z.to(DEV))["loss"].item()
            b.optimizer_step()
            assert la == lb and torch.equal(a.params.flat, b.params.flat)
        if step == 0:
            assert la != ev and math.isfinite(la)
        losses.append(la)
    assert np.mean(losses[-3:]) < np.mean(losses[:3]), losses


def test_lightning_module_drop_in():
    """train_standalone.MatchaLightningModule (the drop-in for train_standalone.py:580-707): validation_step draws
    t and z exactly as the reference does (torch.rand, then torch.randn_like on the device RNG) and matches the
    oracle's losses for those draws; training_step + optimizer.step() update model.MatchaTTS's own parameters."""
    from types import SimpleNamespace

    import train_standalone as TS
    from conftest import DEC, DP, ENC
    sd, x, xl, y, yl, _, _ = _setup(seed=24)
    mod = TS.MatchaLightningModule(178, 1, 64, SimpleNamespace(**ENC), SimpleNamespace(**DEC),
                                   {"solver": "euler", "sigma_min": 1e-4}, SimpleNamespace(**DP),
                                   {"mel_mean": 0.0, "mel_std": 1.0})
    mod.model.load_state_dict(sd)
    mod.to(DEV)
    batch = {"x": x.to(DEV), "x_lengths": xl.to(DEV), "y": y.to(DEV), "y_lengths": yl.to(DEV)}
    torch.manual_seed(99)
    t = torch.rand([3, 1, 1], device=DEV)
    z = torch.randn_like(batch["y"])
    torch.manual_seed(99)
    val = mod.validation_step(batch, 0).item()
    (dur, prior, cfm, _, _), _ = _oracle_grads(sd, x, xl, y, yl, t.view(3).cpu(), z.cpu())
    ref = (dur + prior + cfm).item()
    assert abs(val - ref) <= 1e-4 * abs(ref), (val, ref)
    opt = mod.configure_optimizers()
    w0 = mod.model.state_dict()["decoder.estimator.final_proj.weight"].clone()
    loss = mod.training_step(batch, 0)
    assert math.isfinite(loss.item()) and set(mod.logged) >= {"train/loss", "val/loss"}
    opt.step()
    opt.zero_grad()
    w1 = mod.model.state_dict()["decoder.estimator.final_proj.weight"]
    assert not torch.equal(w0, w1)
    assert torch.equal(w1, mod.trainer().parameters()["decoder.estimator.final_proj.weight"])
    # forward returns maximum_path's [B, T_x, T_y] (train_standalone.py:646, 667)
    assert mod(batch["x"], batch["x_lengths"], batch["y"], batch["y_lengths"])[3].shape == (3, x.shape[1], y.shape[2])


def _lightning(sd, precision="32"):
    from types import SimpleNamespace

    import train_standalone as TS
    from conftest import DEC, DP, ENC
    mod = TS.MatchaLightningModule(178, 1, 64, SimpleNamespace(**ENC), SimpleNamespace(**DEC),
                                   {"solver": "euler", "sigma_min": 1e-4}, SimpleNamespace(**DP),
                                   {"mel_mean": 0.0, "mel_std": 1.0}, precision=precision)
    mod.model.load_state_dict(sd)
    return mod.to(DEV)


@pytest.mark.parametrize("precision", ["32", "16-mixed"])
def test_lightning_module_resume_and_reload(precision):
    """Checkpoint / resume (train_standalone.py:850-857, 882): module.state_dict() + optimizer.state_dict() saved after
    a step and loaded into a FRESH module and optimizer continue bit-identically (the Adam moments, the step count
    and thus the dropout stream come back); a state dict loaded into a live module's .model is what its next step
    trains (the engine's flat parameters are refreshed from it)."""
    sd, x, xl, y, yl, _, _ = _setup(seed=25)
    batch = {"x": x.to(DEV), "x_lengths": xl.to(DEV), "y": y.to(DEV), "y_lengths": yl.to(DEV)}
    a = _lightning(sd, precision)
    opt_a = a.configure_optimizers()
    if precision == "16-mixed":
        # a scale the first steps keep (a skipped step would leave no Adam state to carry), growth after 2 steps
        a.trainer().scaler.update(scale=1024.0, growth_interval=2)
    torch.manual_seed(1)
    a.training_step(batch, 0)
    opt_a.step()
    msd = {k: v.detach().clone() for k, v in a.state_dict().items()}
    osd = opt_a.state_dict()
    assert len(osd["state"]) == len(list(a.parameters())) and float(osd["state"][0]["step"]) == 1.0
    if precision == "16-mixed":  # GradScaler's state rides in the optimizer state (it was dropped)
        assert osd["param_groups"][0]["loss_scaler"] == {"scale": 1024.0, "growth_factor": 2.0, "backoff_factor": 0.5,
                                                         "growth_interval": 2, "_growth_tracker": 1}
    torch.manual_seed(2)
    la = a.training_step(batch, 1).item()
    opt_a.step()
    wa = {k: v.detach().clone() for k, v in a.model.state_dict().items()}
    b = _lightning(sd, precision)
    b.load_state_dict(msd)
    opt_b = b.configure_optimizers()
    opt_b.load_state_dict(osd)
    torch.manual_seed(2)
    lb = b.training_step(batch, 1).item()
    opt_b.step()
    assert la == lb
    if precision == "16-mixed":  # both grew the scale at the second finite step
        assert a.trainer().scaler == b.trainer().scaler and b.trainer().scaler["scale"] == 2048.0
    for k, v in b.model.state_dict().items():
        assert torch.equal(v, wa[k]), k
    # reload into a live module: the next step starts from the loaded weights
    a.model.load_state_dict(sd)
    tp = a.trainer().parameters()
    assert all(torch.equal(tp[k].cpu(), sd[k].float()) for k in tp)


# ----------------------------------------------------------------------------------------- mixed precision
def _autocast_step(sd, x, xl, y, yl, t, z, attn, dt):
    """The reference's own mixed-precision arithmetic: autograd through the oracle on the GPU under
    torch.autocast(dt) on the given alignment; fp16 with GradScaler's rule (loss x 2^16, halved until the gradient
    is finite). -> (losses, unscaled fp32 gradients, the scale that was used)"""
    import oracle.matcha_oracle as O
    S = 65536.0 if dt == torch.float16 else 1.0
    while True:
        params = {k: v.clone().float().to(DEV).requires_grad_(True) for k, v in sd.items()
                  if k.startswith(("encoder.", "decoder.estimator."))}
        with torch.autocast("cuda", dtype=dt):
            dur, prior, cfm, _, _ = O.training_losses(params, *(v.to(DEV) for v in (x, xl, y, yl, t, z)), HP,
                                                      mas=lambda lp, m: attn.to(DEV))
        grads = torch.autograd.grad((dur + prior + cfm) * S, list(params.values()), allow_unused=True)
        g = {k: (gr.float() / S if gr is not None else torch.zeros_like(p)).cpu() for (k, p), gr in
             zip(params.items(), grads)}
        if all(torch.isfinite(v).all() for v in g.values()) or S < 1.0:
            return [float(v) for v in (dur, prior, cfm)], g, S
        S /= 2.0


@pytest.mark.parametrize("precision,dt", [("16-mixed", torch.float16), ("bf16-mixed", torch.bfloat16)])
def test_training_step_mixed_precision_vs_autocast(precision, dt):
    """The whole step in the reference's training precision (train_standalone.py:764, 868: "16-mixed"; and
    "bf16-mixed") at configs[4]'s size (B = 64, T_y = 868), against the fp32 autograd oracle: the alignment is the
    fp32 run's (the log-prior / MAS path stays exact fp32), and the losses and the flat gradient are no further from
    the fp32 oracle than the reference's own mixed arithmetic (the oracle under torch.autocast on the GPU, same
    alignment, fp16 with GradScaler's backoff) is, with a 25 % margin on the flat gradient (measured: 16-mixed 5.5e-3
    vs autocast 1.1e-2, bf16-mixed 1.5e-2 vs 1.9e-2)."""
    from matcha_hip.train import MatchaTrainer
    import oracle.matcha_oracle as O
    sd, x, xl, y, yl, t, z = _configs4_batch(seed=43)
    args = (x.to(DEV), xl.to(DEV), y.to(DEV), yl.to(DEV))
    ref = MatchaTrainer(sd, HP, DEV, dropout=False)
    attn = ref.forward_backward(*args, t=t.to(DEV), z=z.to(DEV))["attn"].cpu()
    del ref
    tr = MatchaTrainer(sd, HP, DEV, dropout=False, precision=precision)
    out = tr.forward_backward(*args, t=t.to(DEV), z=z.to(DEV))
    S = tr.scaler["scale"] if tr.scaler else 1.0
    assert torch.equal(out["attn"].cpu(), attn)
    names = list(tr.grads.names)
    mine = tr.grads.flat.detach().double().cpu() / S
    assert torch.isfinite(mine).all()
    (dur, prior, cfm, _, _), gref = _oracle_grads(sd, x, xl, y, yl, t, z, mas=lambda lp, m: attn)
    flat_ref = torch.cat([gref[n].reshape(-1) for n in names]).double()
    ac_losses, ac_g, ac_S = _autocast_step(sd, x, xl, y, yl, t, z, attn, dt)
    flat_ac = torch.cat([ac_g[n].reshape(-1) for n in names]).double()
    e_mine, e_ac = _rel(mine, flat_ref), _rel(flat_ac, flat_ref)
    l_ref = [float(v) for v in (dur, prior, cfm)]
    l_mine = [float(out[k]) for k in ("dur_loss", "prior_loss", "cfm_loss")]
    print(f"{precision}: flat {e_mine:.3e} vs autocast {e_ac:.3e} (scale {ac_S}); losses "
          f"{[abs(a - b) / abs(b) for a, b in zip(l_mine, l_ref)]} vs {[abs(a - b) / abs(b) for a, b in zip(ac_losses, l_ref)]}")
    assert e_mine <= 1.25 * e_ac, (e_mine, e_ac)
    # a scalar loss is one sample of the rounding noise: no further than 1.5x autocast's error, or within half the
    # operand format's unit roundoff (fp16 2^-12, bf16 2^-9; measured bf16-mixed dur_loss 9.4e-4 vs autocast 7.0e-4)
    floor = 2.0 ** -12 if dt == torch.float16 else 2.0 ** -9
    for a_, c_, r_ in zip(l_mine, ac_losses, l_ref):
        assert abs(a_ - r_) <= max(1.5 * abs(c_ - r_), floor * abs(r_)), (a_, c_, r_)


def test_loss_scaler_skip_backoff_and_growth():
    """GradScaler semantics of "16-mixed" (torch.cuda.amp defaults, Lightning's MixedPrecision plugin): a non-finite
    element anywhere in the gradient (inf or NaN) skips the update — parameters, Adam moments and step count
    untouched — and halves the scale; growth_interval finite steps in a row double it; and each taken step equals
    clip_grad_norm_(5.0) + Adam applied by torch to the unscaled gradient."""
    from matcha_hip.train import MatchaTrainer
    sd, x, xl, y, yl, t, z = _setup(seed=26)
    args = (x.to(DEV), xl.to(DEV), y.to(DEV), yl.to(DEV))
    kw = dict(t=t.to(DEV), z=z.to(DEV))
    tr = MatchaTrainer(sd, HP, DEV, dropout=False, precision="16-mixed")
    tr.scaler.update(scale=1024.0, growth_interval=3)
    for i, bad in enumerate((float("inf"), float("nan"), -float("inf"))):
        tr.forward_backward(*args, **kw)
        p0, m0 = tr.params.flat.clone(), tr.m.clone()
        tr.grads.flat[1000 + 7 * i] = bad
        assert tr.optimizer_step()["skipped"]
        assert tr.scaler["scale"] == 1024.0 / 2 ** (i + 1) and tr.scaler["_growth_tracker"] == 0
        assert tr.step_count == 0 and torch.equal(tr.params.flat, p0) and torch.equal(tr.m, m0)
    tr.scaler["scale"] = 1024.0
    for i in range(3):
        tr.forward_backward(*args, **kw)
        S = tr.scaler["scale"]
        g = {k: v.detach().cpu() / S for k, v in tr.gradients().items()}
        p0 = {k: v.detach().cpu().clone() for k, v in tr.parameters().items()}
        m_ref = [tr.m.cpu().clone(), tr.v.cpu().clone()]
        assert not tr.optimizer_step()["skipped"]
        # torch on the same (unscaled) gradient from the same state: the first step only (fresh Adam moments)
        if i == 0:
            ref = {k: p0[k].clone().requires_grad_(True) for k in tr.grads.names}
            for k, p in ref.items():
                p.grad = g[k].clone()
            norm = torch.nn.utils.clip_grad_norm_(list(ref.values()), 5.0)
            torch.optim.Adam(list(ref.values()), lr=1e-4).step()
            assert abs(tr.last["grad_norm"].item() - norm.item()) <= 1e-5 * norm.item()
            assert max(float((tr.parameters()[k].cpu() - ref[k].detach()).abs().max()) for k in ref) < 5e-7
            assert float(m_ref[0].abs().max()) == 0.0
    assert tr.step_count == 3 and tr.scaler["scale"] == 2048.0 and tr.scaler["_growth_tracker"] == 0


def test_loss_scaler_found_inf_is_per_element():
    """torch's found-inf is per element of the unscaled gradient (torch._amp_foreach_non_finite_check_and_unscale_),
    not a test of the sum of squares: a finite gradient so large that its squared norm overflows fp32 is NOT
    skipped (round-3 verdict) — the clip factor goes to 0, as in clip_grad_norm_, and Adam takes a zero step."""
    from matcha_hip.train import MatchaTrainer
    sd, x, xl, y, yl, t, z = _setup(seed=27)
    tr = MatchaTrainer(sd, HP, DEV, dropout=False, precision="16-mixed")
    tr.scaler.update(scale=1024.0)
    tr.forward_backward(x.to(DEV), xl.to(DEV), y.to(DEV), yl.to(DEV), t=t.to(DEV), z=z.to(DEV))
    tr.grads.flat[5] = 3.0e38  # finite after the unscale; its square overflows
    tr.grads.flat[6] = -3.0e38
    p0 = tr.params.flat.clone()
    out = tr.optimizer_step()
    assert not out["skipped"] and tr.step_count == 1 and tr.scaler["_growth_tracker"] == 1
    assert not math.isfinite(out["grad_norm"].item())
    assert torch.equal(tr.params.flat, p0)  # clip factor 0 -> zero gradient -> Adam's first step moves nothing
