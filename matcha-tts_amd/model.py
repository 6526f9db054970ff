"""Drop-in ``model`` module: ``from model import MatchaTTS`` (main.py:8) on MI355X.

Call surface and state_dict keys are those of the reference ``model.py``
(Lounes78/matcha-tts): ``MatchaTTS(n_vocab, n_spks, spk_emb_dim, encoder_params,
decoder_params, cfm_params, duration_predictor_params)``, ``.synthesize(...) ->
(mel, y_lengths, attn)`` (model.py:1264-1300), plus the upstream-style
``synthesise(...) -> dict`` used by the notebooks.

Everything on the synthesis path runs as hand-written HIP kernels behind the C ABI
(include/matcha_hip.h, ``matcha_hip.runtime``):
  * text encoder + duration predictor (model.py:148-535): ``TextEncoder.forward`` is one
    ``mt_encoder_forward`` call;
  * duration -> alignment index path, CFM Euler/midpoint solver over the U-Net estimator,
    denormalize/crop: ``mt_durations``, ``mt_alignment``, ``mt_cfm_solve``, ``mt_denorm_crop``.
The submodules below only hold parameters under the reference names and shapes (so reference
checkpoints load unchanged); calling one of them directly raises. There is no CPU fallback.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from matcha_hip import runtime as rt


# ======================================================================================
# utilities (model.py:42-125)
# ======================================================================================

def sequence_mask(length: torch.Tensor, max_length: Optional[int] = None) -> torch.Tensor:
    if max_length is None:
        max_length = int(length.max())
    ar = torch.arange(int(max_length), dtype=length.dtype, device=length.device)
    return ar[None, :] < length[:, None]


def fix_len_compatibility(length, num_downsamplings_in_unet: int = 2) -> int:
    """Round up to a multiple of 2**n (host int; model.py:49-55 ends in .item())."""
    f = 2 ** num_downsamplings_in_unet
    return int(math.ceil(int(length) / f) * f)


def denormalize(data, mu, std):
    mu = torch.as_tensor(mu, dtype=data.dtype, device=data.device)
    std = torch.as_tensor(std, dtype=data.dtype, device=data.device)
    return data * std.reshape(-1, 1) + mu.reshape(-1, 1)


def normalize(data, mu, std):
    mu = torch.as_tensor(mu, dtype=data.dtype, device=data.device)
    std = torch.as_tensor(std, dtype=data.dtype, device=data.device)
    return (data - mu.reshape(-1, 1)) / std.reshape(-1, 1)


def _get(p, k, default=None):
    if isinstance(p, dict):
        return p.get(k, default)
    return getattr(p, k, default)


# ======================================================================================
# text encoder parameter containers (state_dict keys of model.py:148-535); TextEncoder.forward is mt_encoder
# ======================================================================================

class _Params(nn.Module):
    """Parameter container of a reference submodule; its arithmetic is a HIP kernel of the owning module."""

    def forward(self, *a, **k):
        raise RuntimeError(f"{type(self).__name__} is evaluated by the HIP path of its owning module "
                           "(TextEncoder.forward / Decoder.forward); it has no forward of its own")


class LayerNorm(_Params):
    """Channel LayerNorm over dim 1 of [B,C,T] (model.py:148-166): gamma, beta."""

    def __init__(self, channels: int, eps: float = 1e-4):
        super().__init__()
        self.channels, self.eps = channels, eps
        self.gamma = nn.Parameter(torch.ones(channels))
        self.beta = nn.Parameter(torch.zeros(channels))


class ConvReluNorm(_Params):
    """Prenet (model.py:171-208): n x (conv(x*mask) -> LayerNorm -> ReLU), zero-init 1x1 proj, residual."""

    def __init__(self, in_channels, hidden_channels, out_channels, kernel_size, n_layers, p_dropout):
        super().__init__()
        self.n_layers = n_layers
        self.conv_layers = nn.ModuleList(
            [nn.Conv1d(in_channels if i == 0 else hidden_channels, hidden_channels, kernel_size,
                       padding=kernel_size // 2) for i in range(n_layers)])
        self.norm_layers = nn.ModuleList([LayerNorm(hidden_channels) for _ in range(n_layers)])
        self.relu_drop = nn.Sequential(nn.ReLU(), nn.Dropout(p_dropout))
        self.proj = nn.Conv1d(hidden_channels, out_channels, 1)
        nn.init.zeros_(self.proj.weight)
        nn.init.zeros_(self.proj.bias)


class DurationPredictor(_Params):
    """model.py:210-235: conv -> relu -> LayerNorm (x2) -> 1x1 -> log-durations."""

    def __init__(self, in_channels, filter_channels, kernel_size, p_dropout):
        super().__init__()
        self.drop = nn.Dropout(p_dropout)
        self.conv_1 = nn.Conv1d(in_channels, filter_channels, kernel_size, padding=kernel_size // 2)
        self.norm_1 = LayerNorm(filter_channels)
        self.conv_2 = nn.Conv1d(filter_channels, filter_channels, kernel_size, padding=kernel_size // 2)
        self.norm_2 = LayerNorm(filter_channels)
        self.proj = nn.Conv1d(filter_channels, 1, 1)


class RotaryPositionalEmebeddings(_Params):
    """RoPE on the first d features (model.py:244-292; name kept for compatibility). No parameters: the
    HIP encoder applies it (rope_kernel) with the theta table of runtime.rope_theta."""

    def __init__(self, d, base: int = 10_000):
        super().__init__()
        self.d, self.base = int(d), base


class MultiHeadAttention(_Params):
    """RoPE multi-head attention with 1x1-conv projections (model.py:294-372)."""

    def __init__(self, channels, out_channels, n_heads, heads_share=True, p_dropout=0.0,
                 proximal_bias=False, proximal_init=False):
        super().__init__()
        assert channels % n_heads == 0, "channels must be divisible by n_heads"
        if proximal_bias:
            raise NotImplementedError("proximal_bias is not used by the reference encoder (model.py:437)")
        self.channels, self.n_heads = channels, n_heads
        self.k_channels = channels // n_heads
        self.conv_q = nn.Conv1d(channels, channels, 1)
        self.conv_k = nn.Conv1d(channels, channels, 1)
        self.conv_v = nn.Conv1d(channels, channels, 1)
        self.query_rotary_pe = RotaryPositionalEmebeddings(self.k_channels * 0.5)
        self.key_rotary_pe = RotaryPositionalEmebeddings(self.k_channels * 0.5)
        self.conv_o = nn.Conv1d(channels, out_channels, 1)
        self.drop = nn.Dropout(p_dropout)
        nn.init.xavier_uniform_(self.conv_q.weight)
        nn.init.xavier_uniform_(self.conv_k.weight)
        if proximal_init:
            with torch.no_grad():
                self.conv_k.weight.copy_(self.conv_q.weight)
                self.conv_k.bias.copy_(self.conv_q.bias)
        nn.init.xavier_uniform_(self.conv_v.weight)


class FFN(_Params):
    """model.py:375-393: conv(x*mask) -> ReLU -> conv(.*mask) * mask."""

    def __init__(self, in_channels, out_channels, filter_channels, kernel_size, p_dropout=0.0):
        super().__init__()
        self.conv_1 = nn.Conv1d(in_channels, filter_channels, kernel_size, padding=kernel_size // 2)
        self.conv_2 = nn.Conv1d(filter_channels, out_channels, kernel_size, padding=kernel_size // 2)
        self.drop = nn.Dropout(p_dropout)


class Encoder(_Params):
    """model.py:396-444: n_layers x (x + MHA -> LayerNorm, x + FFN -> LayerNorm)."""

    def __init__(self, hidden_channels, filter_channels, n_heads, n_layers, kernel_size=1, p_dropout=0.0):
        super().__init__()
        self.n_layers = n_layers
        self.drop = nn.Dropout(p_dropout)
        self.attn_layers = nn.ModuleList(
            [MultiHeadAttention(hidden_channels, hidden_channels, n_heads, p_dropout=p_dropout)
             for _ in range(n_layers)])
        self.norm_layers_1 = nn.ModuleList([LayerNorm(hidden_channels) for _ in range(n_layers)])
        self.ffn_layers = nn.ModuleList(
            [FFN(hidden_channels, hidden_channels, filter_channels, kernel_size, p_dropout=p_dropout)
             for _ in range(n_layers)])
        self.norm_layers_2 = nn.ModuleList([LayerNorm(hidden_channels) for _ in range(n_layers)])


class TextEncoder(nn.Module):
    """model.py:452-535 -> (mu [B,n_feats,Tx], logw [B,1,Tx], x_mask [B,1,Tx])."""

    def __init__(self, encoder_type, encoder_params, duration_predictor_params, n_vocab, n_spks=1,
                 spk_emb_dim=128, precision: str = "fp32"):
        super().__init__()
        self.precision = precision
        self._engines = {}
        self._pk = rt.PackCache()
        self.encoder_type = encoder_type
        self.n_vocab = n_vocab
        self.n_feats = _get(encoder_params, "n_feats")
        self.n_channels = _get(encoder_params, "n_channels")
        self.spk_emb_dim, self.n_spks = spk_emb_dim, n_spks
        self.emb = nn.Embedding(n_vocab, self.n_channels)
        nn.init.normal_(self.emb.weight, 0.0, self.n_channels ** -0.5)
        if _get(encoder_params, "prenet"):
            self.prenet = ConvReluNorm(self.n_channels, self.n_channels, self.n_channels, kernel_size=5,
                                       n_layers=3, p_dropout=0.5)
        else:
            self.prenet = None  # no prenet parameters (the HIP encoder skips the stage)
        width = self.n_channels + (spk_emb_dim if n_spks > 1 else 0)
        self.encoder = Encoder(width, _get(encoder_params, "filter_channels"), _get(encoder_params, "n_heads"),
                               _get(encoder_params, "n_layers"), _get(encoder_params, "kernel_size"),
                               _get(encoder_params, "p_dropout"))
        self.proj_m = nn.Conv1d(width, self.n_feats, 1)
        self.proj_w = DurationPredictor(width, _get(duration_predictor_params, "filter_channels_dp"),
                                        _get(duration_predictor_params, "kernel_size"),
                                        _get(duration_predictor_params, "p_dropout"))

    # ---- HIP plumbing (mt_encoder: the whole forward below is one C-ABI call) ----
    def set_precision(self, precision: str):
        rt.dtype_code(precision)
        self.precision = precision
        return self

    def engine(self) -> rt.EncoderEngine:
        if self.precision not in self._engines:
            enc = self.encoder
            self._engines[self.precision] = rt.EncoderEngine(
                self.n_vocab, self.n_channels, enc.ffn_layers[0].conv_1.out_channels, enc.attn_layers[0].n_heads,
                enc.n_layers, enc.ffn_layers[0].conv_1.kernel_size[0], self.n_spks, self.spk_emb_dim,
                self.proj_w.conv_1.out_channels, self.proj_w.conv_1.kernel_size[0], self.prenet is not None,
                self.precision)
        return self._engines[self.precision]

    def forward(self, x, x_lengths, spks=None):
        """model.py:503-535 on the GPU -> (mu [B,80,Tx], logw [B,1,Tx], x_mask [B,1,Tx]) fp32. An id outside
        [0, n_vocab) raises IndexError, as ``self.emb(x)`` does (model.py:522)."""
        mu, logw, x_mask, oov = self.forward_unchecked(x, x_lengths, spks)
        rt.check_ids(oov)
        return mu, logw, x_mask

    def forward_unchecked(self, x, x_lengths, spks=None):
        """forward without the host sync of the id check: also returns the device flag for ``rt.check_ids``"""
        rt.require_gpu(x, x_lengths, spks, what="TextEncoder.forward")
        if self.n_spks > 1 and spks is None:
            raise ValueError("multi-speaker TextEncoder needs spks [B, spk_emb_dim]")
        eng = self.engine()
        key = (self.precision, str(x.device))
        packed = self._pk.get(key)
        if packed is None:
            sd = self.state_dict(keep_vars=True)
            packed = self._pk.put(key, list(sd.values()), eng.pack(dict(sd), x.device))
        return eng.forward(packed, x, x_lengths, rt.f32c(spks))


# ======================================================================================
# U-Net estimator parameter containers (state_dict keys of model.py:576-962).
# Their arithmetic is the HIP estimator; they have no torch forward of their own.
# ======================================================================================

class LoRACompatibleLinear(nn.Linear):
    pass


class SnakeBeta(_Params):
    def __init__(self, in_features, out_features, alpha=1.0, alpha_trainable=True, alpha_logscale=True):
        super().__init__()
        n = out_features if isinstance(out_features, int) else out_features[0]
        self.proj = nn.Linear(in_features, n)
        self.alpha_logscale = alpha_logscale
        init = torch.zeros(n) if alpha_logscale else torch.ones(n) * alpha
        self.alpha = nn.Parameter(init.clone(), requires_grad=alpha_trainable)
        self.beta = nn.Parameter(init.clone(), requires_grad=alpha_trainable)
        self.no_div_by_zero = 1e-9


class FeedForward(_Params):
    def __init__(self, dim, dim_out=None, mult=4, dropout=0.0, activation_fn="snakebeta", final_dropout=False):
        super().__init__()
        if activation_fn != "snakebeta":
            raise NotImplementedError("the HIP estimator implements the SnakeBeta feed-forward (main.py:74)")
        inner = int(dim * mult)
        self.net = nn.ModuleList([SnakeBeta(dim, inner), nn.Dropout(dropout), nn.Linear(inner, dim_out or dim)])
        if final_dropout:
            self.net.append(nn.Dropout(dropout))


class Attention(_Params):
    def __init__(self, query_dim, heads=8, dim_head=64, dropout=0.0, bias=False, cross_attention_dim=None,
                 upcast_attention=False):
        super().__init__()
        if cross_attention_dim is not None:
            raise NotImplementedError("the reference decoder uses self-attention only (model.py:721-736)")
        if dim_head != 64:
            raise NotImplementedError("the HIP attention kernel is built for head dim 64")
        inner = heads * dim_head
        self.heads, self.scale = heads, dim_head ** -0.5
        self.to_q = nn.Linear(query_dim, inner, bias=bias)
        self.to_k = nn.Linear(query_dim, inner, bias=bias)
        self.to_v = nn.Linear(query_dim, inner, bias=bias)
        self.to_out = nn.ModuleList([nn.Linear(inner, query_dim), nn.Dropout(dropout)])


class BasicTransformerBlock(_Params):
    def __init__(self, dim, num_attention_heads, attention_head_dim, dropout=0.0, activation_fn="snakebeta",
                 attention_bias=False):
        super().__init__()
        if attention_bias:
            raise NotImplementedError("attention_bias=True is not used by the reference decoder")
        self.norm1 = nn.LayerNorm(dim)
        self.attn1 = Attention(dim, num_attention_heads, attention_head_dim, dropout, attention_bias)
        self.norm3 = nn.LayerNorm(dim)
        self.ff = FeedForward(dim, dropout=dropout, activation_fn=activation_fn)


class SinusoidalPosEmb(nn.Module):
    def __init__(self, dim):
        super().__init__()
        assert dim % 2 == 0, "SinusoidalPosEmb requires dim to be even"
        self.dim = dim

    def forward(self, x, scale=1000):   # host helper (model.py:753-762); the HIP path has its own
        x = x.reshape(-1)
        emb = scale * x.unsqueeze(1) * rt.sinus_freq(self.dim).to(x.device).unsqueeze(0)
        return torch.cat((emb.sin(), emb.cos()), dim=-1)


class Block1D(_Params):
    def __init__(self, dim, dim_out, groups=8):
        super().__init__()
        self.block = nn.Sequential(nn.Conv1d(dim, dim_out, 3, padding=1), nn.GroupNorm(groups, dim_out), nn.Mish())


class ResnetBlock1D(_Params):
    def __init__(self, dim, dim_out, time_emb_dim, groups=8):
        super().__init__()
        self.mlp = nn.Sequential(nn.Mish(), nn.Linear(time_emb_dim, dim_out))
        self.block1 = Block1D(dim, dim_out, groups=groups)
        self.block2 = Block1D(dim_out, dim_out, groups=groups)
        self.res_conv = nn.Conv1d(dim, dim_out, 1)


class Downsample1D(_Params):
    def __init__(self, dim):
        super().__init__()
        self.conv = nn.Conv1d(dim, dim, 3, 2, 1)


class Upsample1D(_Params):
    def __init__(self, channels, use_conv_transpose=True, out_channels=None):
        super().__init__()
        if not use_conv_transpose:
            raise NotImplementedError("the reference decoder uses the ConvTranspose1d upsampler")
        self.conv = nn.ConvTranspose1d(channels, out_channels or channels, 4, 2, 1)


class TimestepEmbedding(_Params):
    def __init__(self, in_channels, time_embed_dim, act_fn="silu", out_dim=None):
        super().__init__()
        self.linear_1 = nn.Linear(in_channels, time_embed_dim)
        self.act = nn.SiLU() if act_fn == "silu" else nn.Mish()
        self.linear_2 = nn.Linear(time_embed_dim, out_dim or time_embed_dim)


class Decoder(nn.Module):
    """U-Net velocity estimator (model.py:834-1048). ``forward`` = one HIP estimator evaluation."""

    def __init__(self, in_channels, out_channels, channels=(256, 256), dropout=0.05, attention_head_dim=64,
                 n_blocks=1, num_mid_blocks=2, num_heads=4, time_emb_dim=None, time_mlp_dim=None, ffn_mult=4,
                 precision: str = "fp32", **kwargs):
        super().__init__()
        channels = tuple(channels)
        if channels != (256, 256) or out_channels != 80:
            raise NotImplementedError("the HIP estimator is built for channels=(256,256), n_feats=80 (main.py:68)")
        self.in_channels, self.out_channels = in_channels, out_channels
        self.n_blocks, self.num_mid_blocks, self.num_heads = n_blocks, num_mid_blocks, num_heads
        self.time_embeddings = SinusoidalPosEmb(in_channels)
        tdim = channels[0] * 4
        self.time_mlp = TimestepEmbedding(in_channels, tdim, act_fn="silu")

        def tblocks(dim):
            return nn.ModuleList([BasicTransformerBlock(dim, num_heads, attention_head_dim, dropout, "snakebeta")
                                  for _ in range(n_blocks)])

        self.down_blocks = nn.ModuleList([
            nn.ModuleList([ResnetBlock1D(in_channels, 256, tdim), tblocks(256), Downsample1D(256)]),
            nn.ModuleList([ResnetBlock1D(256, 256, tdim), tblocks(256), nn.Conv1d(256, 256, 3, padding=1)]),
        ])
        self.mid_blocks = nn.ModuleList([nn.ModuleList([ResnetBlock1D(256, 256, tdim), tblocks(256)])
                                         for _ in range(num_mid_blocks)])
        self.up_blocks = nn.ModuleList([
            nn.ModuleList([ResnetBlock1D(512, 256, tdim), tblocks(256), Upsample1D(256, use_conv_transpose=True)]),
            nn.ModuleList([ResnetBlock1D(512, 256, tdim), tblocks(256), nn.Conv1d(256, 256, 3, padding=1)]),
        ])
        self.final_block = Block1D(256, 256)
        self.final_proj = nn.Conv1d(256, out_channels, 1)
        self.precision = precision
        self._engines = {}
        self._pk = rt.PackCache()

    # ---- HIP plumbing ----
    def set_precision(self, precision: str):
        rt.dtype_code(precision)
        self.precision = precision
        return self

    def engine(self) -> rt.DecoderEngine:
        key = self.precision
        if key not in self._engines:
            self._engines[key] = rt.DecoderEngine(self.in_channels, self.num_mid_blocks, self.n_blocks,
                                                  self.num_heads, self.precision)
        return self._engines[key]

    def packed(self, device):
        key = (self.precision, str(device))
        packed = self._pk.get(key)
        if packed is None:
            sd = self.state_dict(keep_vars=True)
            packed = self._pk.put(key, list(sd.values()), self.engine().pack(dict(sd), device))
        return packed

    def forward(self, x, mask, mu, t, spks=None, cond=None):
        """model.py:964-1048 — x, mu [B,80,T], mask [B,1,T], t [B] (or scalar) -> [B,80,T]."""
        rt.require_gpu(x, mask, mu, spks, what="Decoder.forward")
        x, mu, mask, spks = rt.f32c(x), rt.f32c(mu), rt.f32c(mask), rt.f32c(spks)
        t = torch.as_tensor(t, dtype=torch.float32).reshape(-1)
        eng, packed = self.engine(), self.packed(x.device)
        if t.numel() == 1:
            return eng.step(packed, x, mu, mask, spks, float(t[0]))
        # one time per utterance (CFM.compute_loss): one batched call, the times stay on the device
        return eng.step_times(packed, x, mu, mask, spks, t.to(x.device))


# ======================================================================================
# Conditional flow matching (model.py:1063-1162)
# ======================================================================================

class BASECFM(nn.Module):
    def __init__(self, n_feats, cfm_params, n_spks=1, spk_emb_dim=64):
        super().__init__()
        self.n_feats, self.n_spks, self.spk_emb_dim = n_feats, n_spks, spk_emb_dim
        self.solver = _get(cfm_params, "solver", "euler")
        self.sigma_min = _get(cfm_params, "sigma_min", 1e-4)
        self.estimator = None

    @torch.inference_mode()
    def forward(self, mu, mask, n_timesteps, temperature=1.0, spks=None, cond=None, max_valid=None):
        """z = randn_like(mu)*temperature, then the Euler/midpoint loop — one HIP call. max_valid (extension, not
        in the reference signature): the most valid frames of any utterance when the caller knows it (synthesize's
        y_max); it lets the solver prove every utterance padded and use the query-independent attention."""
        rt.require_gpu(mu, mask, spks, what="CFM.forward")
        mu, mask, spks = rt.f32c(mu), rt.f32c(mask), rt.f32c(spks)
        z = torch.randn_like(mu)
        est = self.estimator
        return est.engine().solve(est.packed(mu.device), z, temperature, mu, mask, spks, int(n_timesteps),
                                  self.solver, out=z, max_valid=int(max_valid or 0))

    def compute_loss(self, x1, mask, mu, spks=None, cond=None):
        """model.py:1147-1162 -> (loss, y_t, pred, u_t): t ~ U(0,1) and z ~ N(0,1) per utterance on the
        device, one batched estimator evaluation with a time per utterance (mt_decoder_step_times).
        Forward only (bf16 / fp32 inference estimator, no autograd graph): the training step with its
        hand-written backward is matcha_hip.train.MatchaTrainer (train_standalone.MatchaLightningModule)."""
        b = mu.shape[0]
        t = torch.rand([b, 1, 1], device=mu.device, dtype=mu.dtype)
        z = torch.randn_like(x1)
        y_t = (1 - (1 - self.sigma_min) * t) * z + t * x1
        u_t = x1 - (1 - self.sigma_min) * z
        pred = self.estimator(y_t, mask, mu, t.squeeze(), spks, cond)
        loss = F.mse_loss(pred, u_t, reduction="sum") / (torch.sum(mask) * u_t.shape[1])
        return loss, y_t, pred, u_t


class CFM(BASECFM):
    def __init__(self, n_feats, cfm_params, n_spks=1, spk_emb_dim=64, estimator=None):
        super().__init__(n_feats, cfm_params, n_spks=n_spks, spk_emb_dim=spk_emb_dim)
        if estimator is None:
            raise ValueError("estimator must be provided")
        self.estimator = estimator


# ======================================================================================
# MatchaTTS (model.py:1173-1300)
# ======================================================================================

class MatchaTTS(nn.Module):
    """``precision`` sets the CFM estimator ("fp32" parity mode, "bf16" performance mode). The text encoder and
    duration predictor run in ``encoder_precision``, fp32 by default in BOTH modes: ``ceil(exp(logw))``
    (model.py:1273-1275) flips on a 1-ulp change of logw, so the index path is only bit-exact when logw is the
    reference's fp32 arithmetic; the encoder is < 1 % of the FLOPs."""

    def __init__(self, n_vocab, n_spks, spk_emb_dim, encoder_params, decoder_params, cfm_params,
                 duration_predictor_params, precision: str = "fp32", encoder_precision: str = "fp32"):
        super().__init__()
        self.n_vocab, self.n_spks, self.spk_emb_dim = n_vocab, n_spks, spk_emb_dim
        if n_spks > 1:
            self.spk_emb = nn.Embedding(n_spks, spk_emb_dim)
        self.register_buffer("mel_mean", torch.tensor(0.0))
        self.register_buffer("mel_std", torch.tensor(1.0))
        self.encoder = TextEncoder(_get(encoder_params, "encoder_type"), encoder_params, duration_predictor_params,
                                   n_vocab, n_spks, spk_emb_dim, precision=encoder_precision)
        n_feats = _get(encoder_params, "n_feats")
        dec_in = 2 * n_feats + (spk_emb_dim if n_spks > 1 else 0)
        est = Decoder(in_channels=dec_in, out_channels=n_feats, channels=_get(decoder_params, "channels"),
                      dropout=_get(decoder_params, "dropout"),
                      attention_head_dim=_get(decoder_params, "attention_head_dim"),
                      n_blocks=_get(decoder_params, "n_blocks"), num_mid_blocks=_get(decoder_params, "num_mid_blocks"),
                      num_heads=_get(decoder_params, "num_heads"), act_fn=_get(decoder_params, "act_fn"),
                      precision=precision)
        self.decoder = CFM(n_feats=n_feats, cfm_params=cfm_params, n_spks=n_spks, spk_emb_dim=spk_emb_dim,
                           estimator=est)

    def set_precision(self, precision: str, encoder_precision: str = "fp32"):
        """Estimator: 'fp32' (parity mode, default) or 'bf16' (bf16 MFMA, fp32 accumulate). The text encoder keeps
        fp32 unless ``encoder_precision`` says otherwise (see the class docstring)."""
        self.decoder.estimator.set_precision(precision)
        self.encoder.set_precision(encoder_precision)
        return self

    def forward(self, x, x_lengths, y, y_lengths, spks=None):
        # The reference's MatchaTTS.forward (model.py:1234-1262) is a placeholder: it feeds text-length mu and the
        # text mask to CFM.compute_loss against mel-length y (model.py:1254-1260). The reference trains through
        # MatchaLightningModule.forward (train_standalone.py:623-667) instead, whose drop-in runs on the GPU.
        raise NotImplementedError("train through train_standalone.MatchaLightningModule (the reference's training "
                                  "path, train_standalone.py:580-707); MatchaTTS.forward is a placeholder upstream")

    @torch.inference_mode()
    def synthesize(self, x, x_lengths, n_timesteps, temperature=1.0, spks=None, length_scale=1.0):
        """model.py:1264-1300 -> (mel [B,80,y_max], y_lengths int64 [B], attn [B,1,Tx,T_pad])."""
        rt.require_gpu(x, x_lengths, spks, what="MatchaTTS.synthesize")
        mu, logw, x_mask, oov = self.encoder.forward_unchecked(x, x_lengths, spks)
        w_ceil, cum, y_lengths = rt.durations(logw, x_mask, length_scale)
        # validate the estimator's packed weights now, while the GPU runs the encoder, instead of after the
        # host sync below (nothing between here and the solve can change them)
        est = self.decoder.estimator
        est.packed(x.device)
        est._pk.trust_next((est.precision, str(x.device)))
        try:
            # the reference's host sync (model.py:1278-1281), which also brings back the encoder's out-of-vocabulary
            # flag (one device->host copy for both)
            y_max, bad = rt.fetch_ints(torch.stack((y_lengths.max(), oov[0].to(torch.int64))))
            if bad:
                raise IndexError("index out of range in self (a token id of x lies outside [0, n_vocab))")
            t_pad = fix_len_compatibility(y_max)
            attn, mu_y, y_mask = rt.alignment(cum, y_lengths, t_pad, mu)
            z = self.decoder(mu_y, y_mask, n_timesteps, temperature, spks, cond=None, max_valid=y_max)
        finally:
            est._pk.untrust()
        mel = rt.denorm_crop(z, self.mel_mean, self.mel_std, y_max)
        return mel, y_lengths, attn

    @torch.inference_mode()
    def synthesise(self, x, x_lengths, n_timesteps, temperature=1.0, spks=None, length_scale=1.0):
        """Upstream-Matcha-style alias (notebooks: MOS_audiou_generator.ipynb:294) -> dict."""
        import time
        t0 = time.perf_counter()
        mel, y_lengths, attn = self.synthesize(x, x_lengths, n_timesteps, temperature, spks, length_scale)
        y_max = mel.shape[-1]
        dt = time.perf_counter() - t0
        return {"mel": mel, "mel_lengths": y_lengths, "attn": attn[:, :, :, :y_max],
                "decoder_outputs": normalize(mel, self.mel_mean, self.mel_std),
                "rtf": dt * 22050 / (y_max * 256)}
