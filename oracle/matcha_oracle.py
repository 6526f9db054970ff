"""CPU oracle for the Matcha-TTS synthesis hot path — TEST INFRASTRUCTURE ONLY.

This module is a functional, state-dict-driven restatement of the reference
algorithm (Lounes78/matcha-tts, read-only at /root/reference) for the path

    durations -> alignment/mu_y -> CFM Euler/midpoint ODE over the 1D U-Net
    estimator -> denormalize/crop -> HiFi-GAN v1 Generator -> Denoiser

written from the reference's semantics, NOT copied from it. Every function
cites the reference file:line it restates. It operates on plain dicts of
tensors keyed exactly like the reference ``state_dict`` (so it can be fed the
same synthetic weights as the reference and as the HIP product).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module, and only as the checker / the
reported CPU baseline ("kind": "port"). The product path never calls it.

Parity pinning: the oracle is checked against golden vectors produced by
importing the reference itself in the build container
(``tests/golden/make_golden.py``); see ``tests/test_oracle_golden.py``.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch
import torch.nn.functional as F

Tensor = torch.Tensor
SD = Dict[str, Tensor]


def sub(sd: SD, prefix: str) -> SD:
    """Sub-dict of ``sd`` under ``prefix`` (with the trailing dot stripped)."""
    p = prefix + "."
    return {k[len(p):]: v for k, v in sd.items() if k.startswith(p)}


# ---------------------------------------------------------------------------
# a2: duration -> alignment index path   (model.py:42-76, 1273-1289)
# ---------------------------------------------------------------------------

def sequence_mask(length: Tensor, max_length: int) -> Tensor:
    """model.py:42-46 — ``arange(max) < length[:, None]`` in length's dtype."""
    x = torch.arange(max_length, dtype=length.dtype, device=length.device)
    return x.unsqueeze(0) < length.unsqueeze(1)


def fix_len_compatibility(length: int, num_downsamplings: int = 2) -> int:
    """model.py:49-55 — round up to a multiple of 2**num_downsamplings."""
    f = 2 ** num_downsamplings
    return int(math.ceil(length / f) * f)


def durations(logw: Tensor, x_mask: Tensor, length_scale: float = 1.0):
    """model.py:1273-1275 — w_ceil [B,1,Tx] (float), y_lengths int64 [B]."""
    w = torch.exp(logw) * x_mask * length_scale
    w_ceil = torch.ceil(w)
    y_lengths = torch.clamp_min(torch.sum(w_ceil, [1, 2]), 1).long()
    return w_ceil, y_lengths


def generate_path(duration: Tensor, mask: Tensor) -> Tensor:
    """model.py:64-76 — one-hot monotonic path [B,Tx,Ty].

    path[b,x,j] = ([j < cum[x]] - [j < cum[x-1]]) * mask[b,x,j]
    """
    b, t_x, t_y = mask.shape
    cum = torch.cumsum(duration, 1)
    j = torch.arange(t_y, dtype=cum.dtype)
    upto = (j[None, None, :] < cum[:, :, None]).to(mask.dtype)
    prev = torch.cat([torch.zeros_like(upto[:, :1]), upto[:, :-1]], dim=1)
    return (upto - prev) * mask


def align(logw: Tensor, x_mask: Tensor, mu: Tensor, length_scale: float = 1.0):
    """model.py:1273-1289 — returns (y_lengths, T_pad, y_mask, attn, mu_y)."""
    w_ceil, y_lengths = durations(logw, x_mask, length_scale)
    y_max = int(y_lengths.max())
    t_pad = fix_len_compatibility(y_max)
    y_mask = sequence_mask(y_lengths, t_pad).unsqueeze(1).to(x_mask.dtype)
    attn_mask = x_mask.unsqueeze(-1) * y_mask.unsqueeze(2)
    attn = generate_path(w_ceil.squeeze(1), attn_mask.squeeze(1)).unsqueeze(1)
    mu_y = torch.matmul(attn.squeeze(1).transpose(1, 2), mu.transpose(1, 2)).transpose(1, 2)
    return y_lengths, y_max, t_pad, y_mask, attn, mu_y


# ---------------------------------------------------------------------------
# Text encoder (host PyTorch in the product; restated here so end-to-end
# synthesize can be checked)   model.py:148-535
# ---------------------------------------------------------------------------

def channel_layernorm(x: Tensor, sd: SD, eps: float = 1e-4) -> Tensor:
    """model.py:148-166 — LayerNorm over dim 1 of [B,C,T] with gamma/beta."""
    mean = torch.mean(x, 1, keepdim=True)
    var = torch.mean((x - mean) ** 2, 1, keepdim=True)
    x = (x - mean) * torch.rsqrt(var + eps)
    return x * sd["gamma"].view(1, -1, 1) + sd["beta"].view(1, -1, 1)


def _conv(x, sd, pad=0, **kw):
    return F.conv1d(x, sd["weight"], sd.get("bias"), padding=pad, **kw)


def rope(x: Tensor, d: int, base: int = 10000) -> Tensor:
    """model.py:244-292 — rotary embedding on the first d features of [B,H,T,C]."""
    t = x.shape[2]
    theta = 1.0 / (base ** (torch.arange(0, d, 2).float() / d)).to(x.device)
    idx = torch.arange(t, device=x.device).float()
    it = torch.einsum("n,d->nd", idx, theta)
    it2 = torch.cat([it, it], dim=1)
    cos, sin = it2.cos()[None, None], it2.sin()[None, None]
    xr, xp = x[..., :d], x[..., d:]
    h = d // 2
    neg = torch.cat([-xr[..., h:], xr[..., :h]], dim=-1)
    return torch.cat([xr * cos + neg * sin, xp], dim=-1)


def mha(x: Tensor, sd: SD, n_heads: int, attn_mask: Tensor) -> Tensor:
    """model.py:294-365 — RoPE MHA with 1x1 conv projections, -1e4 key mask."""
    q, k, v = _conv(x, sub(sd, "conv_q")), _conv(x, sub(sd, "conv_k")), _conv(x, sub(sd, "conv_v"))
    b, c, t = q.shape
    kc = c // n_heads

    def heads(z):
        return z.view(b, n_heads, kc, t).transpose(2, 3)

    q, k, v = heads(q), heads(k), heads(v)
    d_rope = int(kc * 0.5)
    q, k = rope(q, d_rope), rope(k, d_rope)
    s = torch.matmul(q, k.transpose(-2, -1)) / math.sqrt(kc)
    s = s.masked_fill(attn_mask == 0, -1e4)
    p = torch.softmax(s, dim=-1)
    o = torch.matmul(p, v).transpose(2, 3).contiguous().view(b, c, t)
    return _conv(o, sub(sd, "conv_o"))


def text_encoder(sd: SD, x: Tensor, x_lengths: Tensor, hp, spks: Optional[Tensor] = None):
    """model.py:503-535 (+ ConvReluNorm :201-208, Encoder :433-444, FFN :388-393,
    DurationPredictor :225-235). Returns mu [B,80,Tx], logw [B,1,Tx], x_mask."""
    n_ch = hp["n_channels"]
    h = F.embedding(x, sd["emb.weight"]) * math.sqrt(n_ch)
    h = h.transpose(1, -1)
    x_mask = sequence_mask(x_lengths, h.size(2)).unsqueeze(1).to(h.dtype)
    # prenet (ConvReluNorm, k=5, 3 layers) model.py:201-208
    org = h
    for i in range(3):
        h = _conv(h * x_mask, sub(sd, f"prenet.conv_layers.{i}"), pad=2)
        h = channel_layernorm(h, sub(sd, f"prenet.norm_layers.{i}"))
        h = torch.relu(h)
    h = (org + _conv(h, sub(sd, "prenet.proj"))) * x_mask
    if hp.get("n_spks", 1) > 1:
        h = torch.cat([h, spks.unsqueeze(-1).repeat(1, 1, h.shape[-1])], dim=1)
    amask = x_mask.unsqueeze(2) * x_mask.unsqueeze(-1)
    ks = hp["kernel_size"]
    for i in range(hp["n_layers"]):
        h = h * x_mask
        y = mha(h, sub(sd, f"encoder.attn_layers.{i}"), hp["n_heads"], amask)
        h = channel_layernorm(h + y, sub(sd, f"encoder.norm_layers_1.{i}"))
        f = _conv(h * x_mask, sub(sd, f"encoder.ffn_layers.{i}.conv_1"), pad=ks // 2)
        f = torch.relu(f)
        f = _conv(f * x_mask, sub(sd, f"encoder.ffn_layers.{i}.conv_2"), pad=ks // 2) * x_mask
        h = channel_layernorm(h + f, sub(sd, f"encoder.norm_layers_2.{i}"))
    h = h * x_mask
    mu = _conv(h, sub(sd, "proj_m")) * x_mask
    dk = hp["dp_kernel_size"]
    h = h.detach()  # model.py:532 — the duration predictor reads a detached copy (matters for autograd only)
    d = _conv(h * x_mask, sub(sd, "proj_w.conv_1"), pad=dk // 2)
    d = channel_layernorm(torch.relu(d), sub(sd, "proj_w.norm_1"))
    d = _conv(d * x_mask, sub(sd, "proj_w.conv_2"), pad=dk // 2)
    d = channel_layernorm(torch.relu(d), sub(sd, "proj_w.norm_2"))
    logw = _conv(d * x_mask, sub(sd, "proj_w.proj")) * x_mask
    return mu, logw, x_mask


# ---------------------------------------------------------------------------
# a5..a11: U-Net estimator (Decoder)   model.py:576-1048
# ---------------------------------------------------------------------------

def mish(x: Tensor) -> Tensor:
    return x * torch.tanh(F.softplus(x))


def sinusoidal_pos_emb(t: Tensor, dim: int, scale: float = 1000) -> Tensor:
    """model.py:747-762."""
    if t.ndim < 1:
        t = t.unsqueeze(0)
    half = dim // 2
    e = math.log(10000) / (half - 1)
    e = torch.exp(torch.arange(half, device=t.device).float() * -e)
    e = scale * t.unsqueeze(1) * e.unsqueeze(0)
    return torch.cat((e.sin(), e.cos()), dim=-1)


def linear(x, sd):
    return F.linear(x, sd["weight"], sd.get("bias"))


def time_mlp(sd: SD, t: Tensor, c_in: int) -> Tensor:
    """model.py:819-832 + :971-972 — [B] -> [B,1024]."""
    e = sinusoidal_pos_emb(t, c_in)
    e = linear(e, sub(sd, "linear_1"))
    e = F.silu(e)
    return linear(e, sub(sd, "linear_2"))


def block1d(sd: SD, x: Tensor, mask: Tensor) -> Tensor:
    """model.py:764-775 — Mish(GroupNorm8(Conv1d k3(x*mask)))*mask."""
    h = F.conv1d(x * mask, sd["block.0.weight"], sd["block.0.bias"], padding=1)
    h = F.group_norm(h, 8, sd["block.1.weight"], sd["block.1.bias"], eps=1e-5)
    return mish(h) * mask


def resnet1d(sd: SD, x: Tensor, mask: Tensor, t_emb: Tensor) -> Tensor:
    """model.py:777-790."""
    h = block1d(sub(sd, "block1"), x, mask)
    h = h + linear(mish(t_emb), sub(sd, "mlp.1")).unsqueeze(-1)
    h = block1d(sub(sd, "block2"), h, mask)
    return h + F.conv1d(x * mask, sd["res_conv.weight"], sd["res_conv.bias"])


def attention(sd: SD, x: Tensor, key_mask: Tensor, heads: int) -> Tensor:
    """model.py:646-705 — self-attention over frames. x [B,T,C], key_mask [B,T].

    Reference quirk kept on purpose (model.py:697): masked keys are filled with
    ``-finfo.min`` = +3.4e38, so a row with any padded key attends uniformly to
    the padded keys only.
    """
    q = linear(x, sub(sd, "to_q"))
    k = linear(x, sub(sd, "to_k"))
    v = linear(x, sub(sd, "to_v"))
    b, t, inner = q.shape
    dh = inner // heads

    def split(z):
        return z.view(b, t, heads, dh).permute(0, 2, 1, 3)

    q, k, v = split(q), split(k), split(v)
    sim = torch.einsum("bhid,bhjd->bhij", q, k) * (dh ** -0.5)
    m = key_mask.unsqueeze(1).unsqueeze(1)
    sim = sim.masked_fill(m == 0, -torch.finfo(sim.dtype).min)
    p = sim.softmax(dim=-1)
    o = torch.einsum("bhij,bhjd->bhid", p, v).permute(0, 2, 1, 3).reshape(b, t, inner)
    return linear(o, sub(sd, "to_out.0"))


def snakebeta_ff(sd: SD, x: Tensor) -> Tensor:
    """model.py:580-644 — Linear 256->1024, SnakeBeta (log-scale), Linear 1024->256."""
    h = linear(x, sub(sd, "net.0.proj"))
    alpha = torch.exp(sd["net.0.alpha"])
    beta = torch.exp(sd["net.0.beta"])
    h = h + (1.0 / (beta + 1e-9)) * torch.pow(torch.sin(h * alpha), 2)
    return linear(h, sub(sd, "net.2"))


def transformer_block(sd: SD, x: Tensor, key_mask: Tensor, heads: int) -> Tensor:
    """model.py:733-744 — x [B,T,C]."""
    n = F.layer_norm(x, (x.shape[-1],), sd["norm1.weight"], sd["norm1.bias"], eps=1e-5)
    x = attention(sub(sd, "attn1"), n, key_mask, heads) + x
    n = F.layer_norm(x, (x.shape[-1],), sd["norm3.weight"], sd["norm3.bias"], eps=1e-5)
    return snakebeta_ff(sub(sd, "ff"), n) + x


def _tblocks(sd: SD, x: Tensor, mask: Tensor, heads: int) -> Tensor:
    x = x.transpose(1, 2)
    km = mask[:, 0, :]
    j = 0
    while f"{j}.norm1.weight" in sd:
        x = transformer_block(sub(sd, str(j)), x, km, heads)
        j += 1
    return x.transpose(1, 2)


def decoder_forward(sd: SD, x: Tensor, mask: Tensor, mu: Tensor, t: Tensor,
                    spks: Optional[Tensor] = None, heads: int = 2, taps: Optional[dict] = None) -> Tensor:
    """model.py:964-1048 — one velocity evaluation. sd = estimator sub-dict. ``taps`` (optional dict) receives the
    block outputs the G2 fixture records with forward hooks (tests/golden/make_golden.py): down0_res, down0_tb,
    mid1_tb, up0_out, up1_tb, all [B,C,T_l]."""
    taps = {} if taps is None else taps
    c_in = sd["time_mlp.linear_1.weight"].shape[1]
    temb = time_mlp(sub(sd, "time_mlp"), t, c_in)
    x = torch.cat([x, mu], dim=1)
    if spks is not None:
        x = torch.cat([x, spks.unsqueeze(-1).expand(-1, -1, x.shape[-1])], dim=1)
    hiddens, masks = [], [mask]
    n_down = sum(1 for k in sd if k.startswith("down_blocks.") and k.endswith(".0.res_conv.weight"))
    for i in range(n_down):
        md = masks[-1]
        x = resnet1d(sub(sd, f"down_blocks.{i}.0"), x, md, temb)
        if i == 0:
            taps["down0_res"] = x
        x = _tblocks(sub(sd, f"down_blocks.{i}.1"), x, md, heads)
        if i == 0:
            taps["down0_tb"] = x
        hiddens.append(x)
        ds = sub(sd, f"down_blocks.{i}.2")
        if i < n_down - 1:   # Downsample1D: Conv1d k3 s2 p1 (model.py:792-798)
            x = F.conv1d(x * md, ds["conv.weight"], ds["conv.bias"], stride=2, padding=1)
        else:                # plain Conv1d k3 p1 (model.py:895-897)
            x = F.conv1d(x * md, ds["weight"], ds["bias"], padding=1)
        masks.append(md[:, :, ::2])
    masks = masks[:-1]
    mm = masks[-1]
    i = 0
    while f"mid_blocks.{i}.0.res_conv.weight" in sd:
        x = resnet1d(sub(sd, f"mid_blocks.{i}.0"), x, mm, temb)
        x = _tblocks(sub(sd, f"mid_blocks.{i}.1"), x, mm, heads)
        taps["mid1_tb"] = x
        i += 1
    n_up = sum(1 for k in sd if k.startswith("up_blocks.") and k.endswith(".0.res_conv.weight"))
    mu_ = None
    for i in range(n_up):
        mu_ = masks.pop()
        skip = hiddens.pop()
        if x.shape[-1] != skip.shape[-1]:
            x = F.interpolate(x, size=skip.shape[-1], mode="nearest")
        x = torch.cat([x, skip], dim=1)
        x = resnet1d(sub(sd, f"up_blocks.{i}.0"), x, mu_, temb)
        x = _tblocks(sub(sd, f"up_blocks.{i}.1"), x, mu_, heads)
        if i == n_up - 1:
            taps["up1_tb"] = x
        us = sub(sd, f"up_blocks.{i}.2")
        if i < n_up - 1:     # Upsample1D: ConvTranspose1d k4 s2 p1 (model.py:800-817)
            x = F.conv_transpose1d(x * mu_, us["conv.weight"], us["conv.bias"], stride=2, padding=1)
            if i == 0:
                taps["up0_out"] = x
        else:
            x = F.conv1d(x * mu_, us["weight"], us["bias"], padding=1)
    x = block1d(sub(sd, "final_block"), x, mu_)
    out = F.conv1d(x * mu_, sd["final_proj.weight"], sd["final_proj.bias"])
    return out * mask


def time_schedule(n_timesteps: int, solver: str = "euler"):
    """The fp32 t values the reference feeds the estimator (model.py:1086-1104)."""
    dt = torch.tensor([1.0 / n_timesteps], dtype=torch.float32)
    ts = []
    for i in range(n_timesteps):
        t = torch.tensor([i / n_timesteps], dtype=torch.float32)
        ts.append(t)
        if solver == "midpoint":
            ts.append(t + dt * 0.5)
    return ts


def cfm_solve(sd: SD, mu: Tensor, mask: Tensor, n_timesteps: int, z: Tensor,
              spks: Optional[Tensor] = None, solver: str = "euler", heads: int = 2) -> Tensor:
    """model.py:1084-1109 with the noise z (= randn_like(mu)*temperature) given."""
    b = z.shape[0]
    dt = torch.tensor([1.0 / n_timesteps] * b, dtype=z.dtype)
    dtb = dt.unsqueeze(1).unsqueeze(1)
    for i in range(n_timesteps):
        t = torch.tensor([i / n_timesteps] * b, dtype=z.dtype)
        pred = decoder_forward(sd, z, mask, mu, t, spks, heads)
        if solver == "euler":
            z = z + pred * dtb
        elif solver == "midpoint":
            zm = z + pred * dtb * 0.5
            pm = decoder_forward(sd, zm, mask, mu, t + dt * 0.5, spks, heads)
            z = z + pm * dtb
        else:
            raise NotImplementedError(solver)
    return z


def denormalize(x: Tensor, mean: Tensor, std: Tensor) -> Tensor:
    """model.py:106-125 — x*std + mean with 0-d (or [C]) buffers broadcast on C."""
    return x * std.reshape(-1, 1) + mean.reshape(-1, 1)


def synthesize(sd: SD, x: Tensor, x_lengths: Tensor, n_timesteps: int, z_fn,
               hp, spks: Optional[Tensor] = None, length_scale: float = 1.0, solver="euler"):
    """model.py:1264-1300. ``z_fn(mu_y)`` supplies randn_like(mu_y)*temperature."""
    mu, logw, x_mask = text_encoder(sub(sd, "encoder"), x, x_lengths, hp, spks)
    y_lengths, y_max, t_pad, y_mask, attn, mu_y = align(logw, x_mask, mu, length_scale)
    z = z_fn(mu_y)
    mel = cfm_solve(sub(sd, "decoder.estimator"), mu_y, y_mask, n_timesteps, z, spks, solver,
                    hp.get("heads", 2))
    mel = denormalize(mel, sd["mel_mean"], sd["mel_std"])[:, :, :y_max]
    return mel, y_lengths, attn


# ---------------------------------------------------------------------------
# a12..a14: HiFi-GAN v1 Generator   hifigan/models.py:14-206
# ---------------------------------------------------------------------------

def fold_weight_norm(g: Tensor, v: Tensor) -> Tensor:
    """torch weight_norm(dim=0) fold used by remove_weight_norm (hifigan/models.py:199-206):
    W = g * v / ||v||, norm over every dim except 0."""
    n = torch.sqrt(torch.sum(v * v, dim=tuple(range(1, v.ndim)), keepdim=True))
    return v * (g / n)


def fold_generator(sd: SD) -> SD:
    """Replace every (weight_g, weight_v) pair by the folded ``weight``."""
    out = {}
    for k, v in sd.items():
        if k.endswith(".weight_g"):
            base = k[: -len("_g")]
            out[base] = fold_weight_norm(v, sd[base + "_v"])
        elif k.endswith(".weight_v"):
            continue
        else:
            out[k] = v
    return out


LRELU_SLOPE = 0.1


def resblock1(sd: SD, x: Tensor, k: int, dil) -> Tensor:
    """hifigan/models.py:90-97 with get_padding (xutils.py:37-38)."""
    for i, d in enumerate(dil):
        xt = F.leaky_relu(x, LRELU_SLOPE)
        xt = F.conv1d(xt, sd[f"convs1.{i}.weight"], sd[f"convs1.{i}.bias"],
                      dilation=d, padding=(k * d - d) // 2)
        xt = F.leaky_relu(xt, LRELU_SLOPE)
        xt = F.conv1d(xt, sd[f"convs2.{i}.weight"], sd[f"convs2.{i}.bias"], padding=(k - 1) // 2)
        x = xt + x
    return x


def resblock2(sd: SD, x: Tensor, k: int, dil) -> Tensor:
    """hifigan/models.py:133-138."""
    for i, d in enumerate(dil):
        xt = F.leaky_relu(x, LRELU_SLOPE)
        xt = F.conv1d(xt, sd[f"convs.{i}.weight"], sd[f"convs.{i}.bias"],
                      dilation=d, padding=(k * d - d) // 2)
        x = xt + x
    return x


def generator_forward(sd: SD, x: Tensor, h) -> Tensor:
    """hifigan/models.py:181-197 on folded weights. x [B,80,T] -> [B,1,256T]."""
    x = F.conv1d(x, sd["conv_pre.weight"], sd["conv_pre.bias"], padding=3)
    nk = len(h["resblock_kernel_sizes"])
    rb = resblock1 if h["resblock"] == "1" else resblock2
    for i, (u, k) in enumerate(zip(h["upsample_rates"], h["upsample_kernel_sizes"])):
        x = F.leaky_relu(x, LRELU_SLOPE)
        x = F.conv_transpose1d(x, sd[f"ups.{i}.weight"], sd[f"ups.{i}.bias"], stride=u,
                               padding=(k - u) // 2)
        xs = None
        for j, (rk, rd) in enumerate(zip(h["resblock_kernel_sizes"], h["resblock_dilation_sizes"])):
            y = rb(sub(sd, f"resblocks.{i * nk + j}"), x, rk, rd)
            xs = y if xs is None else xs + y
        x = xs / nk
    x = F.leaky_relu(x)          # default slope 0.01 (hifigan/models.py:193)
    x = F.conv1d(x, sd["conv_post.weight"], sd["conv_post.bias"], padding=3)
    return torch.tanh(x)


# ---------------------------------------------------------------------------
# a15: Denoiser   hifigan/denoiser.py:11-68
# ---------------------------------------------------------------------------

def _stft_mag_phase(audio: Tensor, n_fft=1024, hop=256, win=1024):
    w = torch.hann_window(win, dtype=audio.dtype)
    s = torch.stft(audio, n_fft=n_fft, hop_length=hop, win_length=win, window=w, return_complex=True)
    s = torch.view_as_real(s)
    return torch.sqrt(s.pow(2).sum(-1)), torch.atan2(s[..., -1], s[..., 0])


def denoiser_bias_spec(gen_sd: SD, h, n_frames: int = 88) -> Tensor:
    """hifigan/denoiser.py:14-60 ('zeros' mode) -> bias_spec [1,513,1]."""
    mel = torch.zeros((1, 80, n_frames), dtype=torch.float32)
    a = generator_forward(gen_sd, mel, h).float().squeeze(0)
    mag, _ = _stft_mag_phase(a)
    return mag[:, :, 0][:, :, None]


def denoise(audio: Tensor, bias_spec: Tensor, strength: float = 0.0005,
            n_fft=1024, hop=256, win=1024) -> Tensor:
    """hifigan/denoiser.py:62-68 — audio [B,L] -> [B, 256*(L//256)]."""
    mag, ang = _stft_mag_phase(audio, n_fft, hop, win)
    mag = torch.clamp(mag - bias_spec * strength, 0.0)
    w = torch.hann_window(win, dtype=audio.dtype)
    return torch.istft(torch.complex(mag * torch.cos(ang), mag * torch.sin(ang)),
                       n_fft=n_fft, hop_length=hop, win_length=win, window=w)


# ---------------------------------------------------------------------------------------------------
# Training side (§8f rank 3): Monotonic Alignment Search, train_standalone.py:280-325 (its pure-Python
# branch, the reference's recurrence with the same-column predecessor path[x-1, y]; float32 numpy
# scalars as the reference runs it). Pinned by tests/golden/g7_mas.npz (make_golden_mas.py ran the
# reference function itself).
# ---------------------------------------------------------------------------------------------------
def maximum_path(neg_cent: Tensor, mask: Tensor) -> Tensor:
    import numpy as np
    value = neg_cent.detach().cpu().numpy().astype(np.float32)
    m = mask.detach().cpu().numpy()
    b, tx_max, ty_max = value.shape
    t_xs = m.sum(axis=1)[:, 0].astype(np.int32)  # train_standalone.py:291-292
    t_ys = m.sum(axis=2)[:, 0].astype(np.int32)
    paths = np.zeros((b, tx_max, ty_max), dtype=np.float32)
    for i in range(b):
        tx, ty = int(t_xs[i]), int(t_ys[i])
        p = np.zeros((tx, ty), dtype=np.float32)  # DP table; unvisited cells stay 0
        v = value[i, :tx, :ty]
        for y in range(ty):  # :306-318
            for x in range(max(0, tx + y - ty), min(tx, y + 1)):
                if x == 0:
                    vp = np.float32(0.0) if y == 0 else p[0, y - 1]
                elif y == 0:
                    vp = p[x - 1, 0]
                else:
                    vp = max(p[x - 1, y], p[x, y - 1])
                p[x, y] = vp + v[x, y]
        index = tx - 1  # backtrack :320-325 (the y = 0 comparison reads a rewritten column: no effect)
        for y in range(ty - 1, -1, -1):
            paths[i, index, y] = 1.0
            if y > 0 and index > 0 and p[index - 1, y - 1] > p[index, y - 1]:
                index -= 1
    return torch.from_numpy(paths)


def maximum_path_diag(neg_cent: Tensor, mask: Tensor) -> Tensor:
    """maximum_path above evaluated one anti-diagonal at a time (numpy vectors instead of Python loops over
    cells), for the configs[4]-sized test. Cell (x, y) reads (x-1, y) and (x, y-1), both on diagonal
    x + y - 1, and only cells of the same valid band (unvisited cells read 0) — the identical float32
    max-then-add per cell, so the table and the path equal maximum_path's (tests/test_oracle_golden.py)."""
    import numpy as np
    value = neg_cent.detach().cpu().numpy().astype(np.float32)
    m = mask.detach().cpu().numpy()
    b, tx_max, ty_max = value.shape
    t_xs = m.sum(axis=1)[:, 0].astype(np.int32)
    t_ys = m.sum(axis=2)[:, 0].astype(np.int32)
    paths = np.zeros((b, tx_max, ty_max), dtype=np.float32)
    for i in range(b):
        tx, ty = int(t_xs[i]), int(t_ys[i])
        p = np.zeros((tx + 1, ty + 1), dtype=np.float32)  # row / column 0 = the "outside" zeros
        v = value[i, :tx, :ty]
        for d in range(tx + ty - 1):
            # the loop's band for column y = d - x: max(0, tx + y - ty) <= x <= min(tx - 1, y)
            xs = np.arange(max(0, d - ty + 1), min(tx - 1, d) + 1)
            ys = d - xs
            keep = (xs >= tx + ys - ty) & (xs <= ys)
            xs, ys = xs[keep], ys[keep]
            if xs.size == 0:
                continue
            up = p[xs, ys + 1]  # (x-1, y): p is shifted by one in both axes
            left = p[xs + 1, ys]  # (x, y-1)
            vp = np.where(xs == 0, np.where(ys == 0, np.float32(0.0), left),
                          np.where(ys == 0, up, np.maximum(up, left)))
            p[xs + 1, ys + 1] = vp + v[xs, ys]
        q = p[1:, 1:]
        index = tx - 1
        for y in range(ty - 1, -1, -1):
            paths[i, index, y] = 1.0
            if y > 0 and index > 0 and q[index - 1, y - 1] > q[index, y - 1]:
                index -= 1
    return torch.from_numpy(paths)


def training_losses(sd: SD, x: Tensor, x_lengths: Tensor, y: Tensor, y_lengths: Tensor, t: Tensor, z: Tensor, hp,
                    sigma_min: float = 1e-4, heads: int = 2, mas=None):
    """train_standalone.py:623-667 (MatchaLightningModule.forward, single speaker, prior_loss on) with
    CFM.compute_loss model.py:1147-1162, duration_loss :79-81; dropout off (eval-mode modules), the noise
    t [B] ~ rand and z ~ randn_like(y) passed in. sd: full model state dict ("encoder.*",
    "decoder.estimator.*"). Differentiable w.r.t. sd's tensors (torch autograd = the gradient oracle).
    Returns (dur_loss, prior_loss, cfm_loss, attn [B,Tx,Ty], log_prior [B,Tx,Ty])."""
    n_feats = y.shape[1]
    mu_x, logw, x_mask = text_encoder(sub(sd, "encoder"), x, x_lengths, hp)
    y_mask = sequence_mask(y_lengths, y.shape[-1]).unsqueeze(1).to(x_mask)
    attn_mask = x_mask.unsqueeze(-1) * y_mask.unsqueeze(2)
    with torch.no_grad():  # :638-647
        const = -0.5 * math.log(2 * math.pi) * n_feats
        factor = -0.5 * torch.ones(mu_x.shape, dtype=mu_x.dtype, device=mu_x.device)
        y_square = torch.matmul(factor.transpose(1, 2), y ** 2)
        y_mu_double = torch.matmul(2.0 * (factor * mu_x).transpose(1, 2), y)
        mu_square = torch.sum(factor * (mu_x ** 2), 1).unsqueeze(-1)
        log_prior = y_square - y_mu_double + mu_square + const
        attn = (mas or maximum_path)(log_prior, attn_mask.squeeze(1)).to(y.device)
    logw_ = torch.log(1e-8 + torch.sum(attn.unsqueeze(1), -1)) * x_mask  # :650-651
    dur_loss = torch.sum((logw - logw_) ** 2) / torch.sum(x_lengths)
    mu_y = torch.matmul(attn.transpose(1, 2), mu_x.transpose(1, 2)).transpose(1, 2)  # :654-655
    tt = t.view(-1, 1, 1)
    y_t = (1 - (1 - sigma_min) * tt) * z + tt * y  # model.py:1150-1162
    u_t = y - (1 - sigma_min) * z
    pred = decoder_forward(sub(sd, "decoder.estimator"), y_t, y_mask, mu_y, t, heads=heads)
    cfm_loss = F.mse_loss(pred, u_t, reduction="sum") / (torch.sum(y_mask) * u_t.shape[1])
    prior_loss = torch.sum(0.5 * ((y - mu_y) ** 2 + math.log(2 * math.pi)) * y_mask)  # :661-663
    prior_loss = prior_loss / (torch.sum(y_mask) * n_feats)
    return dur_loss, prior_loss, cfm_loss, attn, log_prior


# ---------------------------------------------------------------------------------------------------
# §8f rank 4: the log-mel featurizer of the training data path, train_standalone.py:164-201 (identical
# to hifigan/meldataset.py:52-89) and normalize :204-210. librosa (the filterbank's source) is not
# installed here: `librosa_mel_basis` restates librosa.filters.mel (htk=False, norm="slaney", float32)
# element by element, pinned against an independent implementation of the same published algorithm that the
# image carries (transformers 5.15.0 audio_utils.mel_filter_bank, norm / mel_scale "slaney", itself tested
# against librosa upstream): equal to float32 rounding (tests/test_featurizer.py); no librosa output exists in
# the reference. The STFT / magnitude / log / normalisation are the reference's torch ops.
# ---------------------------------------------------------------------------------------------------
def librosa_mel_basis(sr: int, n_fft: int, n_mels: int, fmin: float, fmax: float) -> Tensor:
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, math.log(6.4) / 27.0

    def hz_to_mel(f):
        return min_log_mel + math.log(f / min_log_hz) / logstep if f >= min_log_hz else f / f_sp

    def mel_to_hz(m):
        return min_log_hz * math.exp(logstep * (m - min_log_mel)) if m >= min_log_mel else f_sp * m

    lo, hi = hz_to_mel(float(fmin)), hz_to_mel(float(fmax))
    edges = [mel_to_hz(lo + (hi - lo) * i / (n_mels + 1)) for i in range(n_mels + 2)]
    import numpy as np
    w = np.zeros((n_mels, n_fft // 2 + 1), dtype=np.float32)
    for m in range(n_mels):
        for k in range(n_fft // 2 + 1):
            fk = k * sr / n_fft
            lower = (fk - edges[m]) / (edges[m + 1] - edges[m])
            upper = (edges[m + 2] - fk) / (edges[m + 2] - edges[m + 1])
            w[m, k] = max(0.0, min(lower, upper))
        w[m] = (w[m].astype(np.float64) * (2.0 / (edges[m + 2] - edges[m]))).astype(np.float32)
    return torch.from_numpy(w)


def mel_spectrogram(y: Tensor, basis: Tensor, n_fft=1024, hop=256, win=1024) -> Tensor:
    """train_standalone.py:176-201 with the filterbank given: y [B,L] -> log-mel [B,80,F]."""
    p = (n_fft - hop) // 2
    y = F.pad(y.unsqueeze(1), (p, p), mode="reflect").squeeze(1)
    s = torch.view_as_real(torch.stft(y, n_fft, hop_length=hop, win_length=win, window=torch.hann_window(win),
                                      center=False, pad_mode="reflect", normalized=False, onesided=True,
                                      return_complex=True))
    s = torch.sqrt(s.pow(2).sum(-1) + 1e-9)
    return torch.log(torch.clamp(torch.matmul(basis, s), min=1e-5))
