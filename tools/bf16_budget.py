#!/usr/bin/env python3
"""bf16 error budget of one estimator evaluation (CPU study, no GPU): the oracle's Decoder.forward restated with
bf16 rounding points like the HIP bf16 path's (GEMM operands bf16, fp32 accumulation, every stored tensor rounded),
then with one class of rounding point removed at a time, against the fp32 oracle at the bench shape (B, T from
argv; default B=8 T=728 to keep it quick). Shows which stored tensors carry the error (round-3 verdict item 6).
Usage: python tools/bf16_budget.py [B] [T]"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "matcha-tts_amd"), os.path.join(ROOT, "tests"), ROOT):
    sys.path.insert(0, p)
import oracle.matcha_oracle as O  # noqa: E402
from conftest import make_decoder, rel_rms  # noqa: E402
from matcha_hip import synthetic  # noqa: E402

KEEP = set()  # rounding classes left in fp32


def r(x, cls):
    return x if cls in KEEP else x.bfloat16().float()


def wr(w, wc="w_other"):
    return w if ("weights" in KEEP or wc in KEEP) else w.bfloat16().float()


def conv(x, w, b=None, wc="w_other", **kw):
    y = F.conv1d(r(x, "gemm_in"), wr(w, wc), b, **kw)
    return y


def lin(x, sd, wc="w_other"):
    return F.linear(r(x, "gemm_in"), wr(sd["weight"], wc), sd.get("bias"))


def block1d(sd, x, mask):
    h = conv(x * mask, sd["block.0.weight"], sd["block.0.bias"], wc="w_gnconv", padding=1)
    h = r(h, "conv_out")  # the GroupNorm conv's stored output
    h = F.group_norm(h, 8, sd["block.1.weight"], sd["block.1.bias"], eps=1e-5)
    return O.mish(h) * mask


def resnet1d(sd, x, mask, t_emb):
    h = block1d(O.sub(sd, "block1"), x, mask)
    h = r(h + F.linear(O.mish(t_emb), O.sub(sd, "mlp.1")["weight"], O.sub(sd, "mlp.1")["bias"]).unsqueeze(-1),
          "gn_apply")
    h = block1d(O.sub(sd, "block2"), h, mask)
    return r(h + conv(x * mask, sd["res_conv.weight"], sd["res_conv.bias"], wc="w_res"), "resnet_out")


def attention(sd, x, key_mask, heads):
    q, k, v = (r(lin(x, O.sub(sd, n), "w_qkv"), "qkv") for n in ("to_q", "to_k", "to_v"))
    b, t, inner = q.shape
    dh = inner // heads

    def split(z):
        return z.view(b, t, heads, dh).permute(0, 2, 1, 3)

    q, k, v = split(q), split(k), split(v)
    sim = torch.einsum("bhid,bhjd->bhij", q, k) * (dh ** -0.5)
    m = key_mask.unsqueeze(1).unsqueeze(1)
    sim = sim.masked_fill(m == 0, -torch.finfo(sim.dtype).min)
    p = sim.softmax(dim=-1)
    o = r(torch.einsum("bhij,bhjd->bhid", p, v).permute(0, 2, 1, 3).reshape(b, t, inner), "attn_o")
    return lin(o, O.sub(sd, "to_out.0"), "w_out")


def ff(sd, x):
    h = lin(x, O.sub(sd, "net.0.proj"), "w_ff1")
    alpha, beta = torch.exp(sd["net.0.alpha"]), torch.exp(sd["net.0.beta"])
    h = r(h + (1.0 / (beta + 1e-9)) * torch.pow(torch.sin(h * alpha), 2), "ff_hidden")
    return lin(h, O.sub(sd, "net.2"), "w_ff2")


def tblock(sd, x, km, heads):
    n = F.layer_norm(x, (x.shape[-1],), sd["norm1.weight"], sd["norm1.bias"], eps=1e-5)
    x = r(attention(O.sub(sd, "attn1"), n, km, heads) + x, "resid")
    n = F.layer_norm(x, (x.shape[-1],), sd["norm3.weight"], sd["norm3.bias"], eps=1e-5)
    return r(ff(O.sub(sd, "ff"), n) + x, "resid")


def decoder(sd, x, mask, mu, t, heads=2):
    temb = O.time_mlp(O.sub(sd, "time_mlp"), t, sd["time_mlp.linear_1.weight"].shape[1])
    x = r(torch.cat([x, mu], dim=1), "input")
    hiddens, masks = [], [mask]
    for i in range(2):
        md = masks[-1]
        x = resnet1d(O.sub(sd, f"down_blocks.{i}.0"), x, md, temb)
        x = tblock(O.sub(sd, f"down_blocks.{i}.1.0"), x.transpose(1, 2), md[:, 0], heads).transpose(1, 2)
        hiddens.append(x)
        ds = O.sub(sd, f"down_blocks.{i}.2")
        if i == 0:
            x = r(conv(x * md, ds["conv.weight"], ds["conv.bias"], stride=2, padding=1), "updown")
        else:
            x = r(conv(x * md, ds["weight"], ds["bias"], padding=1), "updown")
        masks.append(md[:, :, ::2])
    masks = masks[:-1]
    mm = masks[-1]
    for i in range(2):
        x = resnet1d(O.sub(sd, f"mid_blocks.{i}.0"), x, mm, temb)
        x = tblock(O.sub(sd, f"mid_blocks.{i}.1.0"), x.transpose(1, 2), mm[:, 0], heads).transpose(1, 2)
    for i in range(2):
        mu_ = masks.pop()
        x = torch.cat([x, hiddens.pop()], dim=1)
        x = resnet1d(O.sub(sd, f"up_blocks.{i}.0"), x, mu_, temb)
        x = tblock(O.sub(sd, f"up_blocks.{i}.1.0"), x.transpose(1, 2), mu_[:, 0], heads).transpose(1, 2)
        us = O.sub(sd, f"up_blocks.{i}.2")
        if i == 0:
            x = r(F.conv_transpose1d(r(x * mu_, "gemm_in"), wr(us["conv.weight"]), us["conv.bias"],
                                     stride=2, padding=1), "updown")
        else:
            x = r(conv(x * mu_, us["weight"], us["bias"], padding=1), "updown")
    x = r(block1d(O.sub(sd, "final_block"), x, mu_), "final")
    return conv(x * mu_, sd["final_proj.weight"], sd["final_proj.bias"], wc="w_final") * mask


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 728
    torch.set_num_threads(8)
    dec = make_decoder(160, "bf16")
    sd = {k: torch.from_numpy(v) for k, v in synthetic.make_state_dict(
        [(k, tuple(v.shape)) for k, v in dec.state_dict().items()], 5).items()}
    rs = np.random.RandomState(B)
    lens = np.clip(np.round(rs.normal(566, 150, B)), 96, T).astype(np.int64)
    lens[0] = T
    g = torch.Generator().manual_seed(B)
    x, mu = torch.randn(B, 80, T, generator=g) * 0.667, torch.randn(B, 80, T, generator=g)
    mask = (torch.arange(T)[None] < torch.from_numpy(lens)[:, None]).float()[:, None]
    t = torch.full((B,), 0.3)
    with torch.inference_mode():
        ref = O.decoder_forward(sd, x, mask, mu * mask, t)
        classes = ["weights", "gemm_in", "conv_out", "gn_apply", "resnet_out", "qkv", "attn_o", "ff_hidden", "resid", "updown",
                   "final", "input"]
        KEEP.clear()
        base = rel_rms(decoder(sd, x, mask, mu * mask, t), ref)
        print(f"all rounding points: rel-RMS {base:.3e}", flush=True)
        for c in classes:
            KEEP.clear()
            KEEP.add(c)
            e = rel_rms(decoder(sd, x, mask, mu * mask, t), ref)
            print(f"  {c:12s} kept fp32: {e:.3e} ({(e - base) / base * 100:+.1f} %)", flush=True)
        for drop, name in ((("gemm_in", "weights"), "only GEMM operands bf16"), (("gemm_in",), "only GEMM inputs bf16"),
                           (("weights",), "only weights bf16"),
                           (("gemm_in", "weights", "conv_out", "resnet_out", "resid"), "storage fp32 except GN conv outputs, resnet outputs, residual stream")):
            KEEP.clear()
            KEEP.update(classes)
            for d in drop:
                KEEP.discard(d)
            e = rel_rms(decoder(sd, x, mask, mu * mask, t), ref)
            print(f"{name}: {e:.3e}", flush=True)
        for wc in ("w_gnconv", "w_res", "w_qkv", "w_out", "w_ff1", "w_ff2", "w_final", "w_other"):
            KEEP.clear()
            KEEP.add(wc)
            e = rel_rms(decoder(sd, x, mask, mu * mask, t), ref)
            print(f"  weights {wc:9s} fp32: {e:.3e} ({(e - base) / base * 100:+.1f} %)", flush=True)
        KEEP.clear()
        KEEP.update(("weights", "resnet_out", "resid"))
        print(f"bf16 except weights, resnet outputs, residual stream: {rel_rms(decoder(sd, x, mask, mu * mask, t), ref):.3e}")
        KEEP.clear()
        KEEP.update(("resnet_out", "resid"))
        print(f"bf16 except resnet outputs, residual stream: {rel_rms(decoder(sd, x, mask, mu * mask, t), ref):.3e}")


if __name__ == "__main__":
    main()
