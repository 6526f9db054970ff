"""CFM training step on the MI355X (§8f rank 3): ``MatchaLightningModule.forward`` / ``training_step`` /
``configure_optimizers`` of train_standalone.py:623-707 with the Trainer settings of :863-874
(gradient_clip_val 5.0, Adam lr 1e-4, DDP gradient averaging).

Every arithmetic op is a HIP kernel of the C ABI (``mtt_*``, csrc/mt_train.hip): GEMMs on exact-fp32 MFMA,
conv1d as im2col + GEMM, GroupNorm / LayerNorm / SnakeBeta / softmax (with the reference's mask quirks) /
RoPE / embedding / dropout forward and backward, the log-prior, Monotonic Alignment Search
(``mt_maximum_path``), the three losses, the global-norm clip and Adam. PyTorch only allocates device
buffers, draws the reference's ``torch.rand`` / ``randn_like`` noise, and (multi-GPU) runs the RCCL
all-reduce. The backward is written out by hand per block (no torch.autograd): each forward returns a
context, each backward takes the output gradient and writes the parameter gradients into ONE flat fp32
buffer. That buffer is laid out in reverse registration order, so the backward fills it front to back;
it is cut into ~25 MB buckets and each bucket's all-reduce is issued (async, RCCL's own stream) as soon as
the backward has produced its last gradient, overlapping the collective with the rest of the backward.
Adam runs once over the flat parameter buffer.

Arithmetic: fp32 (the reference trains under "16-mixed" autocast; this is the higher-precision parity
mode). Multi-speaker conditioning (spk_emb) raises ``NotImplementedError``.
"""
from __future__ import annotations

import math
import re
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from . import runtime as rt
from ._lib import check, lib, ptr, stream_handle

AXPBY, MUL, MISH, MISH_B, SILU, SILU_B, RELU, RELU_B, EXP, SQDIFF, SIN, COS, LOG, RECIP = range(14)
SCALAR = (1, 1, 0, 1, 1, 0)  # broadcast of a one-element b


# ------------------------------------------------------------------------------------------- primitives
def _s(t) -> int:
    return stream_handle(t.device)


def empty(*shape, like) -> torch.Tensor:
    return torch.empty(*shape, dtype=torch.float32, device=like.device)


class _Scratch:
    """grow-only stream-ordered scratch (column-sum partials)"""
    buf: Optional[torch.Tensor] = None

    @classmethod
    def get(cls, n, like):
        if cls.buf is None or cls.buf.numel() < n or cls.buf.device != like.device:
            cls.buf = empty(max(n, 4096), like=like)
        return cls.buf


class _GemmWS(_Scratch):
    """split-K partials of mtt_gemm"""
    buf: Optional[torch.Tensor] = None


# GEMM operand format of the model's conv / linear / attention products (forward and backward): 0 exact fp32
# (precision "32"), 1 fp16 ("16-mixed"), 2 bf16 ("bf16-mixed") — set per step by MatchaTrainer (operand_format).
_OPFMT = [0]
PRECISIONS = {"32": 0, "32-true": 0, "fp32": 0, "16-mixed": 1, "bf16-mixed": 2}


class operand_format:
    """with operand_format(f): the layer products below round their GEMM operands to format f"""

    def __init__(self, fmt: int):
        self.fmt = fmt

    def __enter__(self):
        self.prev, _OPFMT[0] = _OPFMT[0], self.fmt

    def __exit__(self, *exc):
        _OPFMT[0] = self.prev


def gemm(A, B, M, N, K, out, ta=0, tb=0, alpha=1.0, beta=0.0, lda=None, ldb=None, ldc=None, batch=1, sA=0, sB=0,
         sC=0, a_off=0, b_off=0, c_off=0, bias=None, rmask=None, fmt=0):
    """out = (alpha op(A) op(B) + beta out + bias[n]) * rmask[m], row-major; op(A) M x K, op(B) K x N; offsets in
    elements. Long-K / few-tile shapes split K over slices in a workspace (summed in slice order). fmt: operands
    rounded to fp16 (1) / bf16 (2) for 16-bit MFMA with fp32 sums; 0 exact fp32."""
    lda = lda if lda is not None else (M if ta else K)
    ldb = ldb if ldb is not None else (K if tb else N)
    ldc = ldc if ldc is not None else N
    L = lib()
    wsb = L.mtt_gemm_workspace_bytes(M, N, K, batch)
    ws = _GemmWS.get(wsb // 4, out) if wsb else None
    check(L.mtt_gemm_ex(int(fmt), int(ta), int(tb), M, N, K, float(alpha), A.data_ptr() + 4 * a_off, lda, sA,
                        B.data_ptr() + 4 * b_off, ldb, sB, float(beta), out.data_ptr() + 4 * c_off, ldc, sC, batch,
                        ptr(bias), ptr(rmask), ptr(ws), wsb, _s(out)), "gemm")
    return out


def mm(A, B, M, N, K, **kw):
    return gemm(A, B, M, N, K, empty(M, N, like=A), **kw)


def ew(op, out, a=None, b=None, c=None, alpha=1.0, beta=1.0, bc=None, acc=False):
    """out[i] (+)= op(a[i], b[bidx(i)], c[i]) (mtt_ew; a missing operand reads 0); bc = (d0, m0, s0, d1, m1, s1)
    broadcast of b. AXPBY defaults to a + b."""
    n = out.numel()
    d0, m0, s0, d1, m1, s1 = bc if bc is not None else (1, n, 1, 1, 1, 0)
    check(lib().mtt_ew(op, n, ptr(a), ptr(b), ptr(c), out.data_ptr(), float(alpha), float(beta), d0, m0, s0, d1, m1,
                       s1, int(acc), _s(out)), "ew")
    return out


def bc_col(C):  # b[c] over [rows][C]
    return (1, C, 1, 1, 1, 0)


def bc_row(C, rows):  # b[r] over [rows][C]
    return (C, rows, 1, 1, 1, 0)


def bc_bc(B, T, C):  # b[b][c] over [B][T][C]
    return (T * C, B, C, 1, C, 1)


def like_(x):
    return empty(*x.shape, like=x)


def add(a, b, out=None, alpha=1.0, beta=1.0):
    return ew(AXPBY, like_(a) if out is None else out, a, b, alpha=alpha, beta=beta)


def mul_rows(x, m, out=None, alpha=1.0):
    """x [rows][C] * m[rows]"""
    C = x.shape[-1]
    return ew(MUL, like_(x) if out is None else out, x, m, alpha=alpha, bc=bc_row(C, x.numel() // C))


def mul_scalar(x, s, alpha=1.0, out=None):
    """alpha * x * s[0] with s a one-element device tensor"""
    return ew(MUL, like_(x) if out is None else out, x, s, alpha=alpha, bc=SCALAR)


_CONST: Dict[Tuple[str, int], torch.Tensor] = {}


def ones(n, like):
    key = (str(like.device), n)
    if key not in _CONST:
        o = empty(n, like=like)
        ew(AXPBY, o, alpha=0.0)
        _CONST[key] = ew(EXP, o, o)  # exp(0) = 1
    return _CONST[key]


def const(v, like):
    return ew(AXPBY, empty(1, like=like), b=ones(1, like), beta=v, bc=SCALAR)


def eye(n, like):
    key = (str(like.device), -n)
    if key not in _CONST:
        e = empty(n, n, like=like)
        ew(AXPBY, e, alpha=0.0)
        check(lib().mtt_copy_cols(ones(n, like).data_ptr(), 1, 0, e.data_ptr(), n + 1, 0, n, 1, 0, _s(e)), "eye")
        _CONST[key] = e
    return _CONST[key]


def transpose(x, B, R, C):
    """[B][R][C] -> [B][C][R] as op(A) = x^T times I_R (exact: one product by 1, the rest zeros)"""
    out = empty(B, C, R, like=x)
    return gemm(x, eye(R, x), C, R, R, out, ta=1, lda=C, batch=B, sA=R * C, sB=0, sC=R * C)


def cat_cols(a, b):
    """[..][Ca] ++ [..][Cb] along channels"""
    Ca, Cb = a.shape[-1], b.shape[-1]
    rows = a.numel() // Ca
    out = empty(*a.shape[:-1], Ca + Cb, like=a)
    check(lib().mtt_copy_cols(a.data_ptr(), Ca, 0, out.data_ptr(), Ca + Cb, 0, rows, Ca, 0, _s(a)), "cat")
    check(lib().mtt_copy_cols(b.data_ptr(), Cb, 0, out.data_ptr(), Ca + Cb, Ca, rows, Cb, 0, _s(a)), "cat")
    return out


def split_cols(d, Ca):
    C = d.shape[-1]
    rows = d.numel() // C
    a, b = empty(*d.shape[:-1], Ca, like=d), empty(*d.shape[:-1], C - Ca, like=d)
    check(lib().mtt_copy_cols(d.data_ptr(), C, 0, a.data_ptr(), Ca, 0, rows, Ca, 0, _s(d)), "split")
    check(lib().mtt_copy_cols(d.data_ptr(), C, Ca, b.data_ptr(), C - Ca, 0, rows, C - Ca, 0, _s(d)), "split")
    return a, b


def colsum(a, C, out, b=None, seg=None, acc=False):
    rows = a.numel() // C
    seg = rows if seg is None else seg
    scr = _Scratch.get(lib().mtt_colsum_scratch_floats(rows, C, seg), a)
    check(lib().mtt_colsum(a.data_ptr(), ptr(b), rows, C, seg, out.data_ptr(), int(acc), scr.data_ptr(), _s(a)),
          "colsum")
    return out


def total(a, b=None):
    out = empty(1, like=a)
    scr = _Scratch.get(1024, a)
    check(lib().mtt_sum(a.data_ptr(), ptr(b), a.numel(), out.data_ptr(), scr.data_ptr(), _s(a)), "sum")
    return out


def dropout(x, p, seed):
    """identity when p == 0; the backward is the same call on the gradient with the same seed"""
    if p <= 0.0:
        return x
    out = like_(x)
    check(lib().mtt_dropout(x.data_ptr(), x.numel(), float(p), int(seed) & 0xFFFFFFFF, out.data_ptr(), _s(x)),
          "dropout")
    return out


def seq_mask(lengths, T, like):
    B = lengths.shape[0]
    m = empty(B, T, like=like)
    check(lib().mtt_seq_mask(lengths.data_ptr(), B, T, m.data_ptr(), _s(like)), "seq_mask")
    return m


# ---------------------------------------------------------------------------------------- layer blocks
def linear_fwd(x, W, b, rmask=None):
    """x [N][I] -> (x W^T + b) * rmask [N][O] (nn.Linear, Conv1d k=1 with W [O][I][1]; bias and the output row mask
    in the GEMM epilogue)"""
    I = x.shape[-1]
    N, O = x.numel() // I, W.shape[0]
    return mm(x, W, N, O, I, tb=1, bias=b, rmask=rmask, fmt=_OPFMT[0])


def linear_bwd(dy, x, W, gW, gb, need_dx=True):
    I = x.shape[-1]
    N, O = x.numel() // I, W.shape[0]
    gemm(dy, x, O, I, N, gW, ta=1, fmt=_OPFMT[0])
    if gb is not None:
        colsum(dy, O, gb)
    return mm(dy, W, N, I, O, fmt=_OPFMT[0]) if need_dx else None


def conv_fwd(x, W, b, stride=1, pad=0, dil=1, mask=None, out_mask=None):
    """Conv1d of (x * mask): x [B][T][Cin], W [Cout][Cin][k] -> (conv + b) * out_mask [B][Tout][Cout]; the input mask
    is applied while building the columns, bias and output mask in the GEMM epilogue; ctx keeps the columns"""
    B, T, Cin = x.shape
    Cout, _, k = W.shape
    Tout = (T + 2 * pad - dil * (k - 1) - 1) // stride + 1
    cols = empty(B * Tout, Cin * k, like=x)
    check(lib().mtt_im2col(x.data_ptr(), ptr(mask), B, T, Cin, k, stride, pad, dil, Tout, cols.data_ptr(), _s(x)),
          "im2col")
    y = mm(cols, W, B * Tout, Cout, Cin * k, tb=1, bias=b, rmask=out_mask, fmt=_OPFMT[0]).view(B, Tout, Cout)
    return y, (cols, B, T, Cin, k, stride, pad, dil, Tout, mask)


def conv_bwd(dy, ctx, W, gW, gb, need_dx=True):
    """-> d x (times the forward's input mask); weight / bias gradients into gW / gb"""
    cols, B, T, Cin, k, stride, pad, dil, Tout, mask = ctx
    Cout = W.shape[0]
    gemm(dy, cols, Cout, Cin * k, B * Tout, gW, ta=1, fmt=_OPFMT[0])
    if gb is not None:
        colsum(dy, Cout, gb)
    if not need_dx:
        return None
    dcols = mm(dy, W, B * Tout, Cin * k, Cout, fmt=_OPFMT[0])
    dx = empty(B, T, Cin, like=dy)
    check(lib().mtt_col2im(dcols.data_ptr(), ptr(mask), B, T, Cin, k, stride, pad, dil, Tout, dx.data_ptr(), 0,
                           _s(dy)), "col2im")
    return dx


def convT_fwd(x, W, b, stride, pad):
    """ConvTranspose1d: x [B][Tin][Cin], W [Cin][Cout][k] -> [B][Tout][Cout]: the adjoint of the conv with
    weight [Cin][Cout*k] (GEMM to columns, then col2im)"""
    B, Tin, Cin = x.shape
    _, Cout, k = W.shape
    Tout = (Tin - 1) * stride - 2 * pad + k
    dcols = mm(x, W, B * Tin, Cout * k, Cin, fmt=_OPFMT[0])
    y = empty(B, Tout, Cout, like=x)
    check(lib().mtt_col2im(dcols.data_ptr(), None, B, Tout, Cout, k, stride, pad, 1, Tin, y.data_ptr(), 0, _s(x)),
          "col2im")
    if b is not None:
        ew(AXPBY, y, y, b, bc=bc_col(Cout))
    return y, (x, B, Tin, Cin, Cout, k, stride, pad, Tout)


def convT_bwd(dy, ctx, W, gW, gb):
    x, B, Tin, Cin, Cout, k, stride, pad, Tout = ctx
    cols = empty(B * Tin, Cout * k, like=dy)
    check(lib().mtt_im2col(dy.data_ptr(), None, B, Tout, Cout, k, stride, pad, 1, Tin, cols.data_ptr(), _s(dy)),
          "im2col")
    gemm(x, cols, Cin, Cout * k, B * Tin, gW, ta=1, fmt=_OPFMT[0])
    if gb is not None:
        colsum(dy, Cout, gb)
    return mm(cols, W, B * Tin, Cin, Cout * k, tb=1, fmt=_OPFMT[0]).view(B, Tin, Cin)


def ln_fwd(x, g, b, eps):
    C = x.shape[-1]
    rows = x.numel() // C
    y, mean, rstd = like_(x), empty(rows, like=x), empty(rows, like=x)
    check(lib().mtt_layernorm_fwd(x.data_ptr(), g.data_ptr(), b.data_ptr(), rows, C, float(eps), y.data_ptr(),
                                  mean.data_ptr(), rstd.data_ptr(), _s(x)), "layernorm")
    return y, (x, mean, rstd)


def ln_bwd(dy, ctx, g, gg, gb):
    x, mean, rstd = ctx
    C = x.shape[-1]
    rows = x.numel() // C
    dx = like_(x)
    check(lib().mtt_layernorm_bwd(dy.data_ptr(), x.data_ptr(), g.data_ptr(), mean.data_ptr(), rstd.data_ptr(), rows,
                                  C, dx.data_ptr(), _s(x)), "layernorm_bwd")
    xh = ew(AXPBY, like_(x), x, mean, beta=-1.0, bc=bc_row(C, rows))  # xhat = (x - mean) * rstd
    ew(MUL, xh, xh, rstd, bc=bc_row(C, rows))
    colsum(dy, C, gg, b=xh)
    colsum(dy, C, gb)
    return dx


def gn_fwd(x, g, b, G=8, eps=1e-5):
    B, T, C = x.shape
    y, mean, rstd = like_(x), empty(B * G, like=x), empty(B * G, like=x)
    check(lib().mtt_groupnorm_fwd(x.data_ptr(), g.data_ptr(), b.data_ptr(), B, T, C, G, float(eps), y.data_ptr(),
                                  mean.data_ptr(), rstd.data_ptr(), _s(x)), "groupnorm")
    return y, (x, mean, rstd, G)


def gn_bwd(dy, ctx, g, gg, gb):
    x, mean, rstd, G = ctx
    B, T, C = x.shape
    dx, pg, pb = like_(x), empty(B, C, like=x), empty(B, C, like=x)
    check(lib().mtt_groupnorm_bwd(dy.data_ptr(), x.data_ptr(), g.data_ptr(), mean.data_ptr(), rstd.data_ptr(), B, T,
                                  C, G, dx.data_ptr(), pg.data_ptr(), pb.data_ptr(), _s(x)), "groupnorm_bwd")
    colsum(pg, C, gg)
    colsum(pb, C, gb)
    return dx


def act(op, x):
    return ew(op, like_(x), x)


def act_bwd(op_b, x, dy):
    return ew(op_b, like_(x), x, c=dy)


def attention_fwd(q, k, v, kmask, qmask, H, dh, scale, mode, p_drop=0.0, seed=0):
    """q, k, v [B][T][H*dh] -> o [B][T][H*dh]: per head P = softmax(scale q k^T) with the reference's mask
    fill (mode 0 decoder +3.4e38 on masked keys, model.py:697; mode 1 encoder -1e4, model.py:360), dropout on
    P (encoder, model.py:362), O = P v. Batched strided GEMMs over the utterances, one call per head."""
    B, T, D = q.shape
    S = empty(B * H, T, T, like=q)
    for h in range(H):
        gemm(q, k, T, T, dh, S, tb=1, lda=D, ldb=D, ldc=T, batch=B, sA=T * D, sB=T * D, sC=H * T * T, a_off=h * dh,
             b_off=h * dh, c_off=h * T * T, fmt=_OPFMT[0])
    P = empty(B * H, T, T, like=q)
    check(lib().mtt_softmax_fwd(S.data_ptr(), kmask.data_ptr(), ptr(qmask), B * H, H, T, T, float(scale), mode,
                                P.data_ptr(), _s(q)), "softmax")
    del S
    Pd = dropout(P, p_drop, seed)
    o = empty(B, T, D, like=q)
    for h in range(H):
        gemm(Pd, v, T, dh, T, o, lda=T, ldb=D, ldc=D, batch=B, sA=H * T * T, sB=T * D, sC=T * D, a_off=h * T * T,
             b_off=h * dh, c_off=h * dh, fmt=_OPFMT[0])
    return o, (q, k, v, P, Pd, kmask, qmask, H, dh, scale, p_drop, seed)


def attention_bwd(do, ctx):
    q, k, v, P, Pd, kmask, qmask, H, dh, scale, p_drop, seed = ctx
    B, T, D = q.shape
    dPd = empty(B * H, T, T, like=q)
    dq, dk, dv = like_(q), like_(q), like_(q)
    for h in range(H):
        gemm(do, v, T, T, dh, dPd, tb=1, lda=D, ldb=D, ldc=T, batch=B, sA=T * D, sB=T * D, sC=H * T * T,
             a_off=h * dh, b_off=h * dh, c_off=h * T * T, fmt=_OPFMT[0])
        gemm(Pd, do, T, dh, T, dv, ta=1, lda=T, ldb=D, ldc=D, batch=B, sA=H * T * T, sB=T * D, sC=T * D,
             a_off=h * T * T, b_off=h * dh, c_off=h * dh, fmt=_OPFMT[0])
    dP = dropout(dPd, p_drop, seed)
    dS = like_(P)
    check(lib().mtt_softmax_bwd(P.data_ptr(), dP.data_ptr(), kmask.data_ptr(), ptr(qmask), B * H, H, T, T,
                                float(scale), dS.data_ptr(), _s(q)), "softmax_bwd")
    for h in range(H):
        gemm(dS, k, T, dh, T, dq, lda=T, ldb=D, ldc=D, batch=B, sA=H * T * T, sB=T * D, sC=T * D, a_off=h * T * T,
             b_off=h * dh, c_off=h * dh, fmt=_OPFMT[0])
        gemm(dS, q, T, dh, T, dk, ta=1, lda=T, ldb=D, ldc=D, batch=B, sA=H * T * T, sB=T * D, sC=T * D,
             a_off=h * T * T, b_off=h * dh, c_off=h * dh, fmt=_OPFMT[0])
    return dq, dk, dv


def rope_(x, H, dh, d, theta, inverse=False):
    B, T, _ = x.shape
    check(lib().mtt_rope(x.data_ptr(), B, T, H, dh, d, theta.data_ptr(), int(inverse), _s(x)), "rope")
    return x


# ------------------------------------------------------------------------------ gradients + all-reduce
class FlatBuffer:
    """One flat fp32 buffer with a view per named tensor (same order for parameters, gradients, Adam state)."""

    def __init__(self, shapes: List[Tuple[str, Tuple[int, ...]]], device):
        self.names = [n for n, _ in shapes]
        self.spans: List[Tuple[str, int, int]] = []
        o = 0
        for n, s in shapes:
            k = int(math.prod(s))
            self.spans.append((n, o, k))
            o += k
        self.flat = torch.empty(o, dtype=torch.float32, device=device)
        self.view = {n: self.flat[o:o + k].view(s) for (n, o, k), (_, s) in zip(self.spans, shapes)}


class GradBuckets:
    """Bucketed gradient all-reduce overlapped with the backward (torch DDP's reducer, restated for a flat
    buffer the hand-written backward fills in order). Buckets are contiguous ~bucket_bytes ranges of the
    flat gradient; ``mark(name)`` records that a gradient is final and, when it completes its bucket, issues
    that bucket's async all-reduce (SUM; the 1/world average is folded into the clip factor)."""

    def __init__(self, spans: List[Tuple[str, int, int]], flat: torch.Tensor, bucket_bytes: int = 25 << 20,
                 group=None):
        self.flat, self.group = flat, group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self.ranges: List[Tuple[int, int]] = []
        self.members: List[List[str]] = []
        self.bucket_of: Dict[str, int] = {}
        start, nbytes, cur = 0, 0, []
        for i, (n, o, k) in enumerate(spans):
            cur.append(n)
            self.bucket_of[n] = len(self.ranges)
            nbytes += 4 * k
            if nbytes >= bucket_bytes or i == len(spans) - 1:
                self.ranges.append((start, o + k))
                self.members.append(cur)
                start, nbytes, cur = o + k, 0, []
        self.reset()

    def reset(self):
        self.pending = [len(m) for m in self.members]
        self.seen = set()
        self.handles = []
        self.issued: List[int] = []

    def mark(self, name: str):
        if name in self.seen:
            raise RuntimeError(f"gradient {name!r} finalised twice")
        self.seen.add(name)
        b = self.bucket_of[name]
        self.pending[b] -= 1
        if self.pending[b] == 0:
            self.issued.append(b)
            if self.world > 1:
                a, e = self.ranges[b]
                self.handles.append(dist.all_reduce(self.flat[a:e], group=self.group, async_op=True))

    def finish(self):
        missing = [n for n in self.bucket_of if n not in self.seen]
        if missing:
            raise RuntimeError(f"backward produced no gradient for {missing[:5]} (+{max(0, len(missing) - 5)})")
        for h in self.handles:
            h.wait()
        self.handles = []


class Grads:
    """Gradient views of a FlatBuffer under a name prefix; ``done`` forwards to the bucketer."""

    def __init__(self, buf: FlatBuffer, prefix: str = "", buckets: Optional[GradBuckets] = None):
        self.buf, self.prefix, self.buckets = buf, prefix, buckets
        self.view = {n[len(prefix):]: v for n, v in buf.view.items() if n.startswith(prefix)}

    def done(self, *names):
        if self.buckets is not None:
            for n in names:
                self.buckets.mark(self.prefix + n)

    def done_prefix(self, *prefixes):
        self.done(*[n for n in self.view if n.startswith(prefixes)])


# ------------------------------------------------------------------------------------------ the estimator
class EstimatorTrainer:
    """Decoder.forward (model.py:964-1048) with saved activations and its hand-written backward.
    P: estimator-relative reference names -> fp32 device tensors (views of the flat parameter buffer)."""

    def __init__(self, P: Dict[str, torch.Tensor], heads: int = 2, p_drop: float = 0.05):
        self.P, self.H, self.p_drop = P, heads, p_drop
        self.c_cond = P["time_mlp.linear_1.weight"].shape[1]
        self.n_mid = sum(1 for k in P if k.startswith("mid_blocks.") and k.endswith(".0.res_conv.weight"))
        n_down = sum(1 for k in P if k.startswith("down_blocks.") and k.endswith(".0.res_conv.weight"))
        if n_down != 2 or any(re.match(r"(down|mid|up)_blocks\.\d+\.1\.[1-9]", k) for k in P):
            raise NotImplementedError("training step: channels (256, 256) with n_blocks = 1 (the reference config)")
        self.freq = rt.sinus_freq(self.c_cond).to(P["time_mlp.linear_1.weight"].device)

    def block1d_fwd(self, p, x, m):  # model.py:764-775
        P = self.P
        y, cc = conv_fwd(x, P[p + ".block.0.weight"], P[p + ".block.0.bias"], pad=1, mask=m)
        g, gc = gn_fwd(y, P[p + ".block.1.weight"], P[p + ".block.1.bias"])
        return mul_rows(act(MISH, g), m), (m, cc, gc, g)

    def block1d_bwd(self, p, dy, ctx, G):
        P = self.P
        m, cc, gc, g = ctx
        d = act_bwd(MISH_B, g, mul_rows(dy, m))
        d = gn_bwd(d, gc, P[p + ".block.1.weight"], G.view[p + ".block.1.weight"], G.view[p + ".block.1.bias"])
        d = conv_bwd(d, cc, P[p + ".block.0.weight"], G.view[p + ".block.0.weight"], G.view[p + ".block.0.bias"])
        G.done(p + ".block.1.weight", p + ".block.1.bias", p + ".block.0.weight", p + ".block.0.bias")
        return d

    def resnet_fwd(self, p, x, m, mtemb):  # model.py:777-790
        P = self.P
        B, T, _ = x.shape
        h, c1 = self.block1d_fwd(p + ".block1", x, m)
        tb = linear_fwd(mtemb, P[p + ".mlp.1.weight"], P[p + ".mlp.1.bias"])
        Co = tb.shape[-1]
        ew(AXPBY, h, h, tb, bc=bc_bc(B, T, Co))
        h2, c2 = self.block1d_fwd(p + ".block2", h, m)
        xm = mul_rows(x, m)
        r = linear_fwd(xm, P[p + ".res_conv.weight"], P[p + ".res_conv.bias"]).view(B, T, Co)
        return add(h2, r), (x, m, xm, c1, c2)

    def resnet_bwd(self, p, dy, ctx, G, mtemb, dmtemb):
        P = self.P
        x, m, xm, c1, c2 = ctx
        B, T, Cin = x.shape
        dxm = linear_bwd(dy, xm, P[p + ".res_conv.weight"], G.view[p + ".res_conv.weight"],
                         G.view[p + ".res_conv.bias"]).view(B, T, Cin)
        G.done(p + ".res_conv.weight", p + ".res_conv.bias")
        dh = self.block1d_bwd(p + ".block2", dy, c2, G)
        Co = dh.shape[-1]
        dtb = colsum(dh, Co, empty(B, Co, like=dh), seg=T)  # the time bias is broadcast over the frames
        add(dmtemb, linear_bwd(dtb, mtemb, P[p + ".mlp.1.weight"], G.view[p + ".mlp.1.weight"],
                               G.view[p + ".mlp.1.bias"]), out=dmtemb)
        G.done(p + ".mlp.1.weight", p + ".mlp.1.bias")
        dx = self.block1d_bwd(p + ".block1", dh, c1, G)
        return add(dx, mul_rows(dxm, m))

    def tblock_fwd(self, p, x, m, seed):  # BasicTransformerBlock model.py:733-744
        P, H = self.P, self.H
        B, T, C = x.shape
        n1, l1 = ln_fwd(x, P[p + ".norm1.weight"], P[p + ".norm1.bias"], 1e-5)
        q = linear_fwd(n1, P[p + ".attn1.to_q.weight"], None).view(B, T, -1)
        k = linear_fwd(n1, P[p + ".attn1.to_k.weight"], None).view(B, T, -1)
        v = linear_fwd(n1, P[p + ".attn1.to_v.weight"], None).view(B, T, -1)
        dh = q.shape[-1] // H
        o, ac = attention_fwd(q, k, v, m, None, H, dh, dh ** -0.5, 0)
        a = linear_fwd(o, P[p + ".attn1.to_out.0.weight"], P[p + ".attn1.to_out.0.bias"]).view(B, T, C)
        x1 = add(x, dropout(a, self.p_drop, seed))  # to_out[1] Dropout, model.py:668
        n3, l3 = ln_fwd(x1, P[p + ".norm3.weight"], P[p + ".norm3.bias"], 1e-5)
        h = linear_fwd(n3, P[p + ".ff.net.0.proj.weight"], P[p + ".ff.net.0.proj.bias"])
        s = like_(h)
        check(lib().mtt_snake_fwd(h.data_ptr(), P[p + ".ff.net.0.alpha"].data_ptr(), P[p + ".ff.net.0.beta"].data_ptr(),
                                  h.numel(), h.shape[-1], s.data_ptr(), _s(h)), "snake")
        sd = dropout(s, self.p_drop, seed + 1)  # FeedForward net.1 Dropout, model.py:636
        f = linear_fwd(sd, P[p + ".ff.net.2.weight"], P[p + ".ff.net.2.bias"]).view(B, T, C)
        return add(x1, f), (l1, n1, ac, o, l3, n3, h, sd, seed)

    def tblock_bwd(self, p, dy, ctx, G):
        P = self.P
        l1, n1, ac, o, l3, n3, h, sd, seed = ctx
        B, T, C = dy.shape
        dsd = linear_bwd(dy, sd, P[p + ".ff.net.2.weight"], G.view[p + ".ff.net.2.weight"], G.view[p + ".ff.net.2.bias"])
        ds = dropout(dsd, self.p_drop, seed + 1)
        dh, ga, gb = like_(h), like_(h), like_(h)
        check(lib().mtt_snake_bwd(h.data_ptr(), P[p + ".ff.net.0.alpha"].data_ptr(), P[p + ".ff.net.0.beta"].data_ptr(),
                                  ds.data_ptr(), h.numel(), h.shape[-1], dh.data_ptr(), ga.data_ptr(), gb.data_ptr(),
                                  _s(h)), "snake_bwd")
        colsum(ga, h.shape[-1], G.view[p + ".ff.net.0.alpha"])
        colsum(gb, h.shape[-1], G.view[p + ".ff.net.0.beta"])
        dn3 = linear_bwd(dh, n3, P[p + ".ff.net.0.proj.weight"], G.view[p + ".ff.net.0.proj.weight"],
                         G.view[p + ".ff.net.0.proj.bias"]).view(B, T, C)
        dx1 = add(dy, ln_bwd(dn3, l3, P[p + ".norm3.weight"], G.view[p + ".norm3.weight"], G.view[p + ".norm3.bias"]))
        G.done(p + ".ff.net.2.weight", p + ".ff.net.2.bias", p + ".ff.net.0.alpha", p + ".ff.net.0.beta",
               p + ".ff.net.0.proj.weight", p + ".ff.net.0.proj.bias", p + ".norm3.weight", p + ".norm3.bias")
        da = dropout(dx1, self.p_drop, seed)
        do = linear_bwd(da, o, P[p + ".attn1.to_out.0.weight"], G.view[p + ".attn1.to_out.0.weight"],
                        G.view[p + ".attn1.to_out.0.bias"]).view(B, T, -1)
        dq, dk, dv = attention_bwd(do, ac)
        dn1 = linear_bwd(dq, n1, P[p + ".attn1.to_q.weight"], G.view[p + ".attn1.to_q.weight"], None)
        for nm, dd in (("to_k", dk), ("to_v", dv)):
            add(dn1, linear_bwd(dd, n1, P[f"{p}.attn1.{nm}.weight"], G.view[f"{p}.attn1.{nm}.weight"], None), out=dn1)
        dx = add(dx1, ln_bwd(dn1.view(B, T, C), l1, P[p + ".norm1.weight"], G.view[p + ".norm1.weight"],
                             G.view[p + ".norm1.bias"]))
        G.done(p + ".attn1.to_out.0.weight", p + ".attn1.to_out.0.bias", p + ".attn1.to_q.weight",
               p + ".attn1.to_k.weight", p + ".attn1.to_v.weight", p + ".norm1.weight", p + ".norm1.bias")
        return dx

    def forward(self, x, mu, m0, t, seed):
        """x (y_t), mu (mu_y) [B][T][80], m0 (y_mask) [B][T], t [B] -> pred [B][T][80] (masked), ctx"""
        P = self.P
        B, T, F = x.shape
        half = self.c_cond // 2
        # time embedding (model.py:753-762): scale * t first, then times the frequency table
        t1000 = ew(AXPBY, empty(B, 1, like=x), t, alpha=1000.0)
        arg = mm(t1000, self.freq, B, half, 1)
        emb = cat_cols(act(SIN, arg), act(COS, arg))
        h1 = linear_fwd(emb, P["time_mlp.linear_1.weight"], P["time_mlp.linear_1.bias"])  # model.py:819-832
        s1 = act(SILU, h1)
        temb = linear_fwd(s1, P["time_mlp.linear_2.weight"], P["time_mlp.linear_2.bias"])
        mtemb = act(MISH, temb)  # ResnetBlock1D.mlp = Mish -> Linear
        m1 = empty(B, T // 2, like=x)  # masks[-1][:, :, ::2]
        ew(AXPBY, m1, b=m0, beta=1.0, bc=(1, T // 2, 2, T // 2, B, T))
        c = {"emb": emb, "h1": h1, "s1": s1, "temb": temb, "mtemb": mtemb, "m0": m0, "m1": m1}
        h = cat_cols(x, mu)
        h, c["d0r"] = self.resnet_fwd("down_blocks.0.0", h, m0, mtemb)
        h, c["d0t"] = self.tblock_fwd("down_blocks.0.1.0", h, m0, seed + 1)
        h0 = h
        h, c["d0c"] = conv_fwd(h, P["down_blocks.0.2.conv.weight"], P["down_blocks.0.2.conv.bias"], stride=2, pad=1,
                               mask=m0)
        h, c["d1r"] = self.resnet_fwd("down_blocks.1.0", h, m1, mtemb)
        h, c["d1t"] = self.tblock_fwd("down_blocks.1.1.0", h, m1, seed + 3)
        hd1 = h
        h, c["d1c"] = conv_fwd(h, P["down_blocks.1.2.weight"], P["down_blocks.1.2.bias"], pad=1, mask=m1)
        for i in range(self.n_mid):
            h, c[f"m{i}r"] = self.resnet_fwd(f"mid_blocks.{i}.0", h, m1, mtemb)
            h, c[f"m{i}t"] = self.tblock_fwd(f"mid_blocks.{i}.1.0", h, m1, seed + 5 + 2 * i)
        h = cat_cols(h, hd1)
        h, c["u0r"] = self.resnet_fwd("up_blocks.0.0", h, m1, mtemb)
        h, c["u0t"] = self.tblock_fwd("up_blocks.0.1.0", h, m1, seed + 61)
        h, c["u0c"] = convT_fwd(mul_rows(h, m1), P["up_blocks.0.2.conv.weight"], P["up_blocks.0.2.conv.bias"], 2, 1)
        h = cat_cols(h, h0)
        h, c["u1r"] = self.resnet_fwd("up_blocks.1.0", h, m0, mtemb)
        h, c["u1t"] = self.tblock_fwd("up_blocks.1.1.0", h, m0, seed + 63)
        h, c["u1c"] = conv_fwd(h, P["up_blocks.1.2.weight"], P["up_blocks.1.2.bias"], pad=1, mask=m0)
        h, c["fb"] = self.block1d_fwd("final_block", h, m0)
        c["fp_in"] = mul_rows(h, m0)
        return linear_fwd(c["fp_in"], P["final_proj.weight"], P["final_proj.bias"], rmask=m0).view(B, T, F), c

    def backward(self, dpred, c, G):
        """dpred [B][T][80] -> d mu [B][T][80]; parameter gradients into G (estimator-relative names)."""
        P = self.P
        B, T, F = dpred.shape
        m0, m1, mtemb = c["m0"], c["m1"], c["mtemb"]
        dmtemb = ew(AXPBY, like_(mtemb), alpha=0.0)
        d = linear_bwd(mul_rows(dpred, m0), c["fp_in"], P["final_proj.weight"], G.view["final_proj.weight"],
                       G.view["final_proj.bias"])
        G.done("final_proj.weight", "final_proj.bias")
        d = self.block1d_bwd("final_block", mul_rows(d, m0).view(B, T, -1), c["fb"], G)
        d = conv_bwd(d, c["u1c"], P["up_blocks.1.2.weight"], G.view["up_blocks.1.2.weight"],
                     G.view["up_blocks.1.2.bias"])
        G.done("up_blocks.1.2.weight", "up_blocks.1.2.bias")
        d = self.tblock_bwd("up_blocks.1.1.0", d, c["u1t"], G)
        d = self.resnet_bwd("up_blocks.1.0", d, c["u1r"], G, mtemb, dmtemb)
        d, dh0 = split_cols(d, d.shape[-1] // 2)
        d = mul_rows(convT_bwd(d, c["u0c"], P["up_blocks.0.2.conv.weight"], G.view["up_blocks.0.2.conv.weight"],
                               G.view["up_blocks.0.2.conv.bias"]), m1)
        G.done("up_blocks.0.2.conv.weight", "up_blocks.0.2.conv.bias")
        d = self.tblock_bwd("up_blocks.0.1.0", d, c["u0t"], G)
        d = self.resnet_bwd("up_blocks.0.0", d, c["u0r"], G, mtemb, dmtemb)
        d, dhd1 = split_cols(d, d.shape[-1] // 2)
        for i in reversed(range(self.n_mid)):
            d = self.tblock_bwd(f"mid_blocks.{i}.1.0", d, c[f"m{i}t"], G)
            d = self.resnet_bwd(f"mid_blocks.{i}.0", d, c[f"m{i}r"], G, mtemb, dmtemb)
        d = conv_bwd(d, c["d1c"], P["down_blocks.1.2.weight"], G.view["down_blocks.1.2.weight"],
                     G.view["down_blocks.1.2.bias"])
        G.done("down_blocks.1.2.weight", "down_blocks.1.2.bias")
        add(d, dhd1, out=d)
        d = self.tblock_bwd("down_blocks.1.1.0", d, c["d1t"], G)
        d = self.resnet_bwd("down_blocks.1.0", d, c["d1r"], G, mtemb, dmtemb)
        d = conv_bwd(d, c["d0c"], P["down_blocks.0.2.conv.weight"], G.view["down_blocks.0.2.conv.weight"],
                     G.view["down_blocks.0.2.conv.bias"])
        G.done("down_blocks.0.2.conv.weight", "down_blocks.0.2.conv.bias")
        add(d, dh0, out=d)
        d = self.tblock_bwd("down_blocks.0.1.0", d, c["d0t"], G)
        dxin = self.resnet_bwd("down_blocks.0.0", d, c["d0r"], G, mtemb, dmtemb)
        dtemb = act_bwd(MISH_B, c["temb"], dmtemb)
        ds1 = linear_bwd(dtemb, c["s1"], P["time_mlp.linear_2.weight"], G.view["time_mlp.linear_2.weight"],
                         G.view["time_mlp.linear_2.bias"])
        linear_bwd(act_bwd(SILU_B, c["h1"], ds1), c["emb"], P["time_mlp.linear_1.weight"],
                   G.view["time_mlp.linear_1.weight"], G.view["time_mlp.linear_1.bias"], need_dx=False)
        G.done("time_mlp.linear_2.weight", "time_mlp.linear_2.bias", "time_mlp.linear_1.weight",
               "time_mlp.linear_1.bias")
        return split_cols(dxin, F)[1]


# -------------------------------------------------------------------------------------------- the encoder
class EncoderTrainer:
    """TextEncoder.forward (model.py:503-535; ConvReluNorm :201-208, Encoder :433-444, MultiHeadAttention
    :335-365, FFN :388-393, DurationPredictor :225-235) with saved activations and its backward. The
    duration predictor reads a detached copy of the encoder output (:532), so the duration loss trains only
    proj_w. P: TextEncoder-relative names."""

    def __init__(self, P: Dict[str, torch.Tensor], n_layers: int, heads: int, p_drop=0.1, p_prenet=0.5,
                 p_dp=0.1):
        self.P, self.L, self.H = P, n_layers, heads
        self.p, self.p_pre, self.p_dp = p_drop, p_prenet, p_dp
        self.C = P["emb.weight"].shape[1]
        self.dh = self.C // heads
        self.d_rope = int(self.dh * 0.5)
        self.theta = rt.rope_theta(self.dh).to(P["emb.weight"].device)
        self.prenet = "prenet.proj.weight" in P
        self.k = P["encoder.ffn_layers.0.conv_1.weight"].shape[-1]
        self.kd = P["proj_w.conv_1.weight"].shape[-1]

    def cln(self, x, p):  # channel LayerNorm, eps 1e-4 (model.py:148-166)
        return ln_fwd(x, self.P[p + ".gamma"], self.P[p + ".beta"], 1e-4)

    def cln_bwd(self, dy, ctx, p, G):
        return ln_bwd(dy, ctx, self.P[p + ".gamma"], G.view[p + ".gamma"], G.view[p + ".beta"])

    def forward(self, x_ids, x_lengths, seed):
        P, C = self.P, self.C
        B, Tx = x_ids.shape
        dev = P["emb.weight"]
        xm = seq_mask(x_lengths, Tx, dev)
        h = empty(B, Tx, C, like=dev)
        check(lib().mtt_embed_fwd(x_ids.data_ptr(), B * Tx, dev.data_ptr(), C, math.sqrt(C), h.data_ptr(), _s(dev)),
              "embed")
        c = {"ids": x_ids, "xm": xm, "seed": seed}
        if self.prenet:
            org, pre = h, []
            for i in range(3):
                W = P[f"prenet.conv_layers.{i}.weight"]
                y, cc = conv_fwd(h, W, P[f"prenet.conv_layers.{i}.bias"], pad=W.shape[-1] // 2, mask=xm)
                n, lc = self.cln(y, f"prenet.norm_layers.{i}")
                h = dropout(act(RELU, n), self.p_pre, seed + i)
                pre.append((cc, lc, n))
            c["pre"], c["pre_last"] = pre, h
            h = mul_rows(add(org, linear_fwd(h, P["prenet.proj.weight"], P["prenet.proj.bias"]).view(B, Tx, C)), xm)
        layers = []
        for i in range(self.L):
            a, s = f"encoder.attn_layers.{i}", seed + 10 + 4 * i
            hm = mul_rows(h, xm)
            q = linear_fwd(hm, P[a + ".conv_q.weight"], P[a + ".conv_q.bias"]).view(B, Tx, C)
            k = linear_fwd(hm, P[a + ".conv_k.weight"], P[a + ".conv_k.bias"]).view(B, Tx, C)
            v = linear_fwd(hm, P[a + ".conv_v.weight"], P[a + ".conv_v.bias"]).view(B, Tx, C)
            rope_(q, self.H, self.dh, self.d_rope, self.theta)
            rope_(k, self.H, self.dh, self.d_rope, self.theta)
            o, ac = attention_fwd(q, k, v, xm, xm, self.H, self.dh, 1.0 / math.sqrt(self.dh), 1, self.p, s)
            y = linear_fwd(o, P[a + ".conv_o.weight"], P[a + ".conv_o.bias"]).view(B, Tx, C)
            h1, l1 = self.cln(add(hm, dropout(y, self.p, s + 1)), f"encoder.norm_layers_1.{i}")
            f = f"encoder.ffn_layers.{i}"
            f1, c1 = conv_fwd(h1, P[f + ".conv_1.weight"], P[f + ".conv_1.bias"], pad=self.k // 2, mask=xm)
            rd = dropout(act(RELU, f1), self.p, s + 2)
            f2, c2 = conv_fwd(rd, P[f + ".conv_2.weight"], P[f + ".conv_2.bias"], pad=self.k // 2, mask=xm,
                              out_mask=xm)
            h, l2 = self.cln(add(h1, dropout(f2, self.p, s + 3)), f"encoder.norm_layers_2.{i}")
            layers.append((hm, ac, o, l1, c1, f1, c2, l2))
        c["layers"] = layers
        hm = mul_rows(h, xm)
        c["hm"] = hm
        mu = linear_fwd(hm, P["proj_m.weight"], P["proj_m.bias"], rmask=xm).view(B, Tx, -1)
        d1, dc1 = conv_fwd(hm, P["proj_w.conv_1.weight"], P["proj_w.conv_1.bias"], pad=self.kd // 2)
        n1, dl1 = self.cln(act(RELU, d1), "proj_w.norm_1")
        d2, dc2 = conv_fwd(dropout(n1, self.p_dp, seed + 50), P["proj_w.conv_2.weight"], P["proj_w.conv_2.bias"],
                           pad=self.kd // 2, mask=xm)
        n2, dl2 = self.cln(act(RELU, d2), "proj_w.norm_2")
        n2m = mul_rows(dropout(n2, self.p_dp, seed + 51), xm)
        logw = linear_fwd(n2m, P["proj_w.proj.weight"], P["proj_w.proj.bias"], rmask=xm).view(B, Tx)
        c["dp"] = (d1, dc1, dl1, d2, dc2, dl2, n2m)
        return mu, logw, xm, c

    def backward(self, dmu, dlogw, c, G):
        """dmu [B][Tx][80], dlogw [B][Tx] -> parameter gradients into G (TextEncoder-relative names)."""
        P, C = self.P, self.C
        xm, seed = c["xm"], c["seed"]
        B, Tx, _ = dmu.shape
        # duration predictor: its input is detached, nothing flows back into the encoder
        d1, dc1, dl1, d2, dc2, dl2, n2m = c["dp"]
        dn2m = linear_bwd(mul_rows(dlogw.view(B, Tx, 1), xm), n2m, P["proj_w.proj.weight"],
                          G.view["proj_w.proj.weight"], G.view["proj_w.proj.bias"]).view(B, Tx, -1)
        dn2 = dropout(mul_rows(dn2m, xm), self.p_dp, seed + 51)
        dd2 = act_bwd(RELU_B, d2, self.cln_bwd(dn2, dl2, "proj_w.norm_2", G))
        dn1 = conv_bwd(dd2, dc2, P["proj_w.conv_2.weight"], G.view["proj_w.conv_2.weight"],
                       G.view["proj_w.conv_2.bias"])
        dd1 = act_bwd(RELU_B, d1, self.cln_bwd(dropout(dn1, self.p_dp, seed + 50), dl1, "proj_w.norm_1", G))
        conv_bwd(dd1, dc1, P["proj_w.conv_1.weight"], G.view["proj_w.conv_1.weight"], G.view["proj_w.conv_1.bias"],
                 need_dx=False)
        G.done_prefix("proj_w.")
        dh = linear_bwd(mul_rows(dmu, xm), c["hm"], P["proj_m.weight"], G.view["proj_m.weight"],
                        G.view["proj_m.bias"]).view(B, Tx, C)
        dh = mul_rows(dh, xm)
        G.done("proj_m.weight", "proj_m.bias")
        for i in reversed(range(self.L)):
            a, s, f = f"encoder.attn_layers.{i}", seed + 10 + 4 * i, f"encoder.ffn_layers.{i}"
            hm, ac, o, l1, c1, f1, c2, l2 = c["layers"][i]
            ds = self.cln_bwd(dh, l2, f"encoder.norm_layers_2.{i}", G)  # d(h1 + drop(ffn))
            df2 = mul_rows(dropout(ds, self.p, s + 3), xm)
            drd = conv_bwd(df2, c2, P[f + ".conv_2.weight"], G.view[f + ".conv_2.weight"], G.view[f + ".conv_2.bias"])
            df1 = act_bwd(RELU_B, f1, dropout(drd, self.p, s + 2))
            dh1 = add(ds, conv_bwd(df1, c1, P[f + ".conv_1.weight"], G.view[f + ".conv_1.weight"],
                                   G.view[f + ".conv_1.bias"]))
            ds1 = self.cln_bwd(dh1, l1, f"encoder.norm_layers_1.{i}", G)  # d(hm + drop(attn))
            do = linear_bwd(dropout(ds1, self.p, s + 1), o, P[a + ".conv_o.weight"], G.view[a + ".conv_o.weight"],
                            G.view[a + ".conv_o.bias"]).view(B, Tx, C)
            dq, dk, dv = attention_bwd(do, ac)
            rope_(dq, self.H, self.dh, self.d_rope, self.theta, inverse=True)
            rope_(dk, self.H, self.dh, self.d_rope, self.theta, inverse=True)
            dhm = ds1
            for nm, dd in (("conv_q", dq), ("conv_k", dk), ("conv_v", dv)):
                dhm = add(dhm, linear_bwd(dd, hm, P[f"{a}.{nm}.weight"], G.view[f"{a}.{nm}.weight"],
                                          G.view[f"{a}.{nm}.bias"]).view(B, Tx, C))
            dh = mul_rows(dhm, xm)
            G.done_prefix(a + ".", f + ".", f"encoder.norm_layers_1.{i}.", f"encoder.norm_layers_2.{i}.")
        if self.prenet:
            dorg = dh  # h = (org + proj(r)) * m, dh already masked
            drd = linear_bwd(dh, c["pre_last"], P["prenet.proj.weight"], G.view["prenet.proj.weight"],
                             G.view["prenet.proj.bias"]).view(B, Tx, C)
            for i in reversed(range(3)):
                cc, lc, n = c["pre"][i]
                dn = act_bwd(RELU_B, n, dropout(drd, self.p_pre, seed + i))
                dy = self.cln_bwd(dn, lc, f"prenet.norm_layers.{i}", G)
                drd = conv_bwd(dy, cc, P[f"prenet.conv_layers.{i}.weight"], G.view[f"prenet.conv_layers.{i}.weight"],
                               G.view[f"prenet.conv_layers.{i}.bias"])
            dh = add(dorg, drd)
            G.done_prefix("prenet.")
        check(lib().mtt_embed_bwd(c["ids"].data_ptr(), B * Tx, dh.data_ptr(), P["emb.weight"].shape[0], C,
                                  math.sqrt(C), G.view["emb.weight"].data_ptr(), _s(dh)), "embed_bwd")
        G.done("emb.weight")


# --------------------------------------------------------------------------------------------- the step
def log_prior(mu_x, y_btc):
    """train_standalone.py:639-644: -0.5 |y_j|^2 + <mu_i, y_j> - 0.5 |mu_i|^2 - 0.5 log(2 pi) F, [B][Tx][Ty]"""
    B, Tx, F = mu_x.shape
    Ty = y_btc.shape[1]
    lp = empty(B, Tx, Ty, like=mu_x)
    gemm(mu_x, y_btc, Tx, Ty, F, lp, tb=1, batch=B, sA=Tx * F, sB=Ty * F, sC=Tx * Ty)
    one = ones(F, mu_x)
    mu_sq = mm(ew(MUL, like_(mu_x), mu_x, mu_x), one, B * Tx, 1, F, alpha=-0.5)
    y_sq = mm(ew(MUL, like_(y_btc), y_btc, y_btc), one, B * Ty, 1, F, alpha=-0.5)
    ew(AXPBY, y_sq, y_sq, const(-0.5 * math.log(2 * math.pi) * F, mu_x), bc=SCALAR)
    ew(AXPBY, lp, lp, mu_sq, bc=bc_row(Ty, B * Tx))
    ew(AXPBY, lp, lp, y_sq, bc=(1, Ty, 1, Tx * Ty, B, Ty))
    return lp


class MatchaTrainer:
    """Training step of the Matcha-TTS acoustic model (single speaker) on the GPU.

    state: the MatchaTTS state dict ("encoder.*", "decoder.estimator.*" reference names); hp: encoder
    hyper-parameters (n_layers, n_heads). Parameters, gradients and Adam moments live in flat fp32 buffers
    on ``device``; ``parameters()`` / ``gradients()`` return reference-named views."""

    def __init__(self, state: Dict[str, torch.Tensor], hp: dict, device, lr: float = 1e-4, sigma_min: float = 1e-4,
                 prior_loss: bool = True, dropout: bool = True, grad_clip: float = 5.0, heads: int = 2,
                 process_group=None, bucket_bytes: int = 25 << 20, seed: int = 0,
                 p_dropout: Optional[Dict[str, float]] = None, precision: str = "32"):
        """p_dropout: the configs' rates {"encoder", "duration_predictor", "decoder"} (train_standalone.py:772-800:
        encoder_params.p_dropout, duration_predictor_params.p_dropout, decoder_params.dropout; defaults 0.1 / 0.1 /
        0.05); the prenet's 0.5 is fixed in the reference (model.py:481). On a DDP group (world > 1) rank 0's
        parameters are broadcast at construction, as DistributedDataParallel does when it wraps the module.

        precision: Lightning's Trainer precision (train_standalone.py:868 trains with "16-mixed"). "32": exact fp32
        MFMA everywhere. "16-mixed": every conv / linear / attention product, forward and backward, on fp16-rounded
        operands (16-bit MFMA, fp32 sums), with torch.cuda.amp.GradScaler's dynamic loss scale (init 2^16, x0.5
        and the step skipped on an inf / NaN gradient, x2 after 2000 finite steps); "bf16-mixed": bf16 operands, no
        scaler. Activations, norms, softmax, losses and the Adam state stay fp32 in every mode; the log-prior / MAS
        products and the alignment GEMMs (0/1 attn) stay exact fp32."""
        if int(hp.get("n_spks", 1)) > 1:
            raise NotImplementedError("multi-speaker training (spk_emb conditioning) is not built")
        names = [k for k, v in state.items() if k.startswith(("encoder.", "decoder.estimator."))
                 and torch.is_floating_point(v)]
        self.names = names
        shapes = [(k, tuple(state[k].shape)) for k in reversed(names)]  # the backward fills the buffer in order
        dev = torch.device(device)
        self.params, self.grads = FlatBuffer(shapes, dev), FlatBuffer(shapes, dev)
        for k in names:
            self.params.view[k].copy_(state[k].detach().to(torch.float32))
        self.m = torch.zeros_like(self.params.flat)
        self.v = torch.zeros_like(self.params.flat)
        self.buckets = GradBuckets(self.grads.spans, self.grads.flat, bucket_bytes, process_group)
        self.world, self.group = self.buckets.world, process_group
        if self.world > 1:  # DDP's start-up broadcast: every rank begins from rank 0's weights
            dist.broadcast(self.params.flat, src=dist.get_global_rank(process_group, 0) if process_group else 0,
                           group=process_group)
        enc_P = {k[len("encoder."):]: v for k, v in self.params.view.items() if k.startswith("encoder.")}
        est_P = {k[len("decoder.estimator."):]: v for k, v in self.params.view.items()
                 if k.startswith("decoder.estimator.")}
        self.enc = EncoderTrainer(enc_P, int(hp["n_layers"]), int(hp["n_heads"]))
        self.est = EstimatorTrainer(est_P, heads)
        pd = {"encoder": 0.1, "duration_predictor": 0.1, "decoder": 0.05}
        pd.update(p_dropout or {})
        self.p_dropout = pd
        self.set_dropout(dropout)
        self.lr, self.sigma_min, self.prior, self.clip = lr, sigma_min, prior_loss, grad_clip
        self.step_count, self.seed, self.calls = 0, seed, 0
        self.last: Dict[str, torch.Tensor] = {}
        if precision not in PRECISIONS:
            raise ValueError(f"precision {precision!r}: one of {sorted(PRECISIONS)}")
        self.precision, self.opfmt = precision, PRECISIONS[precision]
        # torch.cuda.amp.GradScaler defaults (Lightning's MixedPrecision plugin for "16-mixed")
        self.scaler = {"scale": 65536.0, "growth_factor": 2.0, "backoff_factor": 0.5, "growth_interval": 2000,
                       "_growth_tracker": 0} if self.opfmt == 1 else None

    def set_dropout(self, enabled: bool):
        """train (True: the configured rates, train_standalone.py:775-800, and the prenet's fixed 0.5, model.py:481)
        or eval (False: identity) dropout"""
        on = 1.0 if enabled else 0.0
        pd = self.p_dropout
        self.enc.p, self.enc.p_pre, self.enc.p_dp = pd["encoder"] * on, 0.5 * on, pd["duration_predictor"] * on
        self.est.p_drop = pd["decoder"] * on
        self.dropout = bool(enabled)
        return self

    def parameters(self) -> Dict[str, torch.Tensor]:
        return dict(self.params.view)

    @torch.no_grad()
    def load_parameters(self, state: Dict[str, torch.Tensor]):
        """overwrite the flat parameters from reference-named tensors (a checkpoint loaded into the module);
        the Adam moments and the step count are kept"""
        for k in self.names:
            self.params.view[k].copy_(state[k].detach().to(device=self.params.flat.device, dtype=torch.float32))

    def optimizer_state(self) -> Dict[str, object]:
        """Adam's exp_avg / exp_avg_sq (flat, parameter order of ``self.grads.names``), step count and lr"""
        st = {"exp_avg": self.m, "exp_avg_sq": self.v, "step": self.step_count, "lr": self.lr, "calls": self.calls}
        if self.scaler is not None:  # GradScaler.state_dict() keys
            st["scaler"] = dict(self.scaler)
        return st

    @torch.no_grad()
    def load_optimizer_state(self, st: Dict[str, object]):
        self.m.copy_(st["exp_avg"])
        self.v.copy_(st["exp_avg_sq"])
        self.step_count = int(st["step"])
        # the dropout stream's position (one per forward_backward call; a step the scaler skipped still advanced it)
        self.calls = int(st["calls"]) if st.get("calls") is not None else self.step_count
        self.lr = float(st.get("lr", self.lr))
        if self.scaler is not None and st.get("scaler"):
            self.scaler.update({k: st["scaler"][k] for k in self.scaler if k in st["scaler"]})

    def gradients(self) -> Dict[str, torch.Tensor]:
        return dict(self.grads.view)

    def forward_backward(self, x, x_lengths, y, y_lengths, t: Optional[torch.Tensor] = None,
                         z: Optional[torch.Tensor] = None, backward: bool = True):
        """train_standalone.py:623-667 + the backward of dur + prior + cfm. x int64 [B][Tx], y [B][80][Ty]
        (Ty % 4 == 0, the collate's fix_len_compatibility), lengths int64 [B]; t [B] / z [B][80][Ty] default to
        the reference's draws (torch.rand, torch.randn_like). Leaves the all-reduced (summed over ranks)
        gradients in the flat buffer; returns the losses as device scalars. backward=False: losses only
        (validation_step)."""
        rt.require_gpu(x, y, what="MatchaTrainer")
        lo, hi = (int(v) for v in torch.aminmax(x))  # nn.Embedding raises on an out-of-vocabulary id
        n_vocab = self.params.view["encoder.emb.weight"].shape[0]
        if lo < 0 or hi >= n_vocab:
            raise IndexError(f"token id out of range [0, {n_vocab}): min {lo}, max {hi}")
        B, Tx = x.shape
        F, Ty = y.shape[1], y.shape[2]
        if Ty % 4:
            raise ValueError(f"mel length {Ty} must be a multiple of 4 (fix_len_compatibility)")
        x = x.to(torch.int64).contiguous()
        xl, yl = x_lengths.to(torch.int64).contiguous(), y_lengths.to(torch.int64).contiguous()
        y = y.to(torch.float32).contiguous()
        if t is None:
            t = torch.rand([B, 1, 1], device=y.device, dtype=y.dtype)
        if z is None:
            z = torch.randn_like(y)
        t, z = t.reshape(B).to(torch.float32).contiguous(), z.to(torch.float32).contiguous()
        # dropout streams advance per call (a step the loss scaler skips does not reuse its masks)
        seed = ((self.seed * 1000003 + self.calls) * 256) & 0xFFFFFFFF
        self.calls += 1
        self.buckets.reset()
        with operand_format(self.opfmt):
            return self._forward_backward(x, xl, y, yl, t, z, seed, backward)

    def _forward_backward(self, x, xl, y, yl, t, z, seed, backward):
        B, Tx = x.shape
        F, Ty = y.shape[1], y.shape[2]
        S = self.scaler["scale"] if self.scaler else 1.0  # the loss scale seeds the backward
        # ---- forward
        mu_x, logw, xm, ectx = self.enc.forward(x, xl, seed)
        ym = seq_mask(yl, Ty, y)
        y_btc, z_btc = transpose(y, B, F, Ty), transpose(z, B, F, Ty)
        lp = log_prior(mu_x, y_btc)
        attn = empty(B, Tx, Ty, like=y)
        t_xs, t_ys = xl.clamp(max=Tx).to(torch.int32), yl.clamp(max=Ty).to(torch.int32)
        ws = rt._Workspace.get(lib().mt_maximum_path_workspace_bytes(B, Tx, Ty), y.device)
        check(lib().mt_maximum_path(lp.data_ptr(), t_xs.data_ptr(), t_ys.data_ptr(), B, Tx, Ty, attn.data_ptr(),
                                    ws.data_ptr(), ws.numel(), _s(y)), "maximum_path")
        mu_y = empty(B, Ty, F, like=y)
        gemm(attn, mu_x, Ty, F, Tx, mu_y, ta=1, batch=B, sA=Tx * Ty, sB=Tx * F, sC=Ty * F)
        # flow matching (model.py:1147-1162)
        coef = ew(AXPBY, empty(B, like=y), t, ones(1, y), alpha=-(1.0 - self.sigma_min), beta=1.0, bc=SCALAR)
        bcb = (Ty * F, B, 1, 1, 1, 0)
        y_t = add(ew(MUL, like_(z_btc), z_btc, coef, bc=bcb), ew(MUL, like_(y_btc), y_btc, t, bc=bcb))
        u_t = add(y_btc, z_btc, beta=-(1.0 - self.sigma_min))
        pred, dctx = self.est.forward(y_t, mu_y, ym, t, seed + 128)
        n80 = mul_scalar(total(ym), ones(1, y), alpha=float(F))
        inv_n80 = ew(RECIP, empty(1, like=y), n80, alpha=1.0)
        diff = add(pred, u_t, beta=-1.0)
        cfm = mul_scalar(total(diff, diff), inv_n80)
        dpred = mul_scalar(diff, inv_n80, alpha=2.0 * S)
        # prior loss (train_standalone.py:661-663)
        ymu = add(y_btc, mu_y, beta=-1.0)
        if self.prior:
            e = ew(AXPBY, like_(ymu), ew(MUL, like_(ymu), ymu, ymu), const(math.log(2 * math.pi), y), bc=SCALAR)
            prior = mul_scalar(total(mul_rows(e, ym, alpha=0.5)), inv_n80)
        else:
            prior = ew(AXPBY, empty(1, like=y), alpha=0.0)
        # duration loss (train_standalone.py:650-651, 336-339)
        lw_ = ew(LOG, empty(B, Tx, like=y), mm(attn, ones(Ty, y), B * Tx, 1, Ty), alpha=1e-8)
        ew(MUL, lw_, lw_, xm)
        dl = add(logw, lw_, beta=-1.0)
        inv_nx = ew(RECIP, empty(1, like=y), total(xm), alpha=1.0)
        dur = mul_scalar(total(dl, dl), inv_nx)
        dlogw = mul_scalar(dl, inv_nx, alpha=2.0 * S)
        if not backward:
            loss = add(add(dur, prior), cfm)
            self.last = {"loss": loss, "dur_loss": dur, "prior_loss": prior, "cfm_loss": cfm, "attn": attn,
                         "log_prior": lp}
            return self.last
        # ---- backward
        dmu_y = self.est.backward(dpred, dctx, Grads(self.grads, "decoder.estimator.", self.buckets))
        if self.prior:
            add(dmu_y, mul_scalar(mul_rows(ymu, ym, alpha=-S), inv_n80), out=dmu_y)
        dmu_x = empty(B, Tx, F, like=y)
        gemm(attn, dmu_y, Tx, F, Ty, dmu_x, batch=B, sA=Tx * Ty, sB=Ty * F, sC=Tx * F)
        self.enc.backward(dmu_x, dlogw, ectx, Grads(self.grads, "encoder.", self.buckets))
        self.buckets.finish()
        loss = add(add(dur, prior), cfm)
        self.last = {"loss": loss, "dur_loss": dur, "prior_loss": prior, "cfm_loss": cfm, "attn": attn,
                     "log_prior": lp}
        return self.last

    def optimizer_step(self):
        """gradient_clip_val 5.0 (norm of the world-averaged gradient) then torch.optim.Adam (lr, defaults).
        "16-mixed" runs Lightning's MixedPrecision sequence: GradScaler.unscale_ (the summed, loss-scaled buffer times
        1 / (world * scale) in place, with torch's per-element found-inf check on the values as stored, before the
        multiply), the clip on the unscaled gradient, then GradScaler.step / update: a non-finite element skips the
        update and halves the scale, ``growth_interval`` finite steps in a row double it. The found-inf flag is read on the host, as
        GradScaler.step does (``found_inf.item()``); the all-reduced buffer is the same on every rank."""
        g = self.grads.flat
        scale = empty(2, like=g)
        if self.scaler is not None:
            sc = self.scaler
            found = empty(1, like=g)
            check(lib().mtt_unscale(g.data_ptr(), g.numel(), 1.0 / (self.world * sc["scale"]), found.data_ptr(),
                                    _Scratch.get(1024, g).data_ptr(), _s(g)), "unscale")
            sumsq = total(g, g)
            if found.item() != 0.0:
                sc["scale"] *= sc["backoff_factor"]
                sc["_growth_tracker"] = 0
                self.last["grad_norm"] = sumsq.sqrt()
                self.last["skipped"] = True
                return self.last
            sc["_growth_tracker"] += 1
            if sc["_growth_tracker"] == sc["growth_interval"]:
                sc["scale"] *= sc["growth_factor"]
                sc["_growth_tracker"] = 0
            inv = 1.0  # already unscaled and averaged
        else:
            sumsq = total(g, g)
            inv = 1.0 / self.world  # the buffer holds the sum over ranks; the average folds into the clip factor
        self.step_count += 1
        check(lib().mtt_clip_factor(sumsq.data_ptr(), float(self.clip), inv, scale.data_ptr(), scale[1:].data_ptr(),
                                    _s(g)), "clip_factor")
        check(lib().mtt_adam(self.params.flat.data_ptr(), g.data_ptr(), self.m.data_ptr(), self.v.data_ptr(), g.numel(),
                             scale.data_ptr(), float(self.lr), 0.9, 0.999, 1e-8, self.step_count, _s(g)), "adam")
        self.last["grad_norm"] = scale[1:]
        self.last["skipped"] = False
        return self.last

    def training_step(self, batch: dict):
        """train_standalone.py:669-685: batch with x, x_lengths, y, y_lengths -> losses (device scalars)."""
        if batch.get("spks") is not None:
            raise NotImplementedError("multi-speaker training (spk_emb conditioning) is not built")
        self.forward_backward(batch["x"], batch["x_lengths"], batch["y"], batch["y_lengths"])
        return self.optimizer_step()
