"""Generate golden vectors by running the REFERENCE (read-only /root/reference).

Run in the build container only (the GPU box has no /root/reference):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Weights come from the committed recipe ``matcha_hip/synthetic.py`` (seeded per
key), so only inputs/outputs and (key, shape) manifests are stored. Noise ``z``
is injected by patching ``torch.randn_like`` while the reference CFM runs.
Fixtures: G1 duration/index path, G2 one Decoder.forward (+
per-block intermediates), G3 CFM Euler n=4 and midpoint n=2, G4 Generator (+
per-stage outputs, weight-norm fold), G5 Denoiser, G6 end-to-end synthesize.
The script also checks the oracle restatement against every fixture.
"""
from __future__ import annotations

import importlib.util
import json
import os
import sys
from types import SimpleNamespace

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.dont_write_bytecode = True
sys.path.insert(0, REF)
sys.path.insert(0, REPO)

import model as ref_model                                    # noqa: E402  (reference)
from hifigan import models as ref_hifi                       # noqa: E402  (reference)
from hifigan.config import v1 as ref_v1                      # noqa: E402
from hifigan.env import AttrDict                             # noqa: E402
from hifigan.denoiser import Denoiser as RefDenoiser         # noqa: E402

_spec = importlib.util.spec_from_file_location(
    "synthetic", os.path.join(REPO, "matcha-tts_amd", "matcha_hip", "synthetic.py"))
synthetic = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(synthetic)
from oracle import matcha_oracle as O                        # noqa: E402

torch.set_num_threads(8)
SEED = 1234

ENC = dict(encoder_type="RoPE Encoder", n_feats=80, n_channels=192, filter_channels=768,
           n_heads=2, n_layers=6, kernel_size=3, p_dropout=0.1, prenet=True)
DEC = dict(channels=(256, 256), dropout=0.05, attention_head_dim=64, n_blocks=1,
           num_mid_blocks=2, num_heads=2, act_fn="snakebeta")
DP = dict(filter_channels_dp=256, kernel_size=3, p_dropout=0.1)
CFM = {"solver": "euler", "sigma_min": 1e-4}


def load_synth(module: torch.nn.Module, seed=SEED, **kw):
    sd = module.state_dict()
    w = synthetic.make_state_dict([(k, tuple(v.shape)) for k, v in sd.items()], seed, **kw)
    module.load_state_dict({k: torch.from_numpy(v) for k, v in w.items()})
    module.eval()
    return {k: torch.from_numpy(v) for k, v in w.items()}


def manifest(module):
    return json.dumps([[k, list(v.shape)] for k, v in module.state_dict().items()])


def save(name, **arrs):
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **{k: (np.asarray(v) if not torch.is_tensor(v) else v.detach().cpu().numpy())
                                 for k, v in arrs.items()})
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.0f} KiB)")


def close(a, b, tol, what):
    err = (a - b).abs().max().item()
    ok = err <= tol
    print(f"  oracle vs reference {what}: max|d|={err:.3e} {'OK' if ok else 'FAIL'}")
    assert ok, what


def make_matcha(n_spks=1):
    return ref_model.MatchaTTS(n_vocab=178, n_spks=n_spks, spk_emb_dim=64,
                               encoder_params=SimpleNamespace(**ENC),
                               decoder_params=SimpleNamespace(**DEC), cfm_params=dict(CFM),
                               duration_predictor_params=SimpleNamespace(**DP))


def g1():
    rs = np.random.RandomState(11)
    B, Tx = 3, 40
    xl = torch.tensor([40, 31, 17])
    x_mask = O.sequence_mask(xl, Tx).unsqueeze(1).float()
    logw = torch.from_numpy(rs.normal(0.6, 0.7, (B, 1, Tx)).astype(np.float32)) * x_mask
    mu = torch.from_numpy(rs.standard_normal((B, 80, Tx)).astype(np.float32)) * x_mask
    out = {}
    for i, ls in enumerate([1.0, 0.85]):
        w = torch.exp(logw) * x_mask * ls
        w_ceil = torch.ceil(w)
        yl = torch.clamp_min(torch.sum(w_ceil, [1, 2]), 1).long()
        ymax = yl.max()
        tp = ref_model.fix_len_compatibility(ymax)
        ym = ref_model.sequence_mask(yl, tp).unsqueeze(1).to(x_mask.dtype)
        am = x_mask.unsqueeze(-1) * ym.unsqueeze(2)
        attn = ref_model.generate_path(w_ceil.squeeze(1), am.squeeze(1)).unsqueeze(1)
        mu_y = torch.matmul(attn.squeeze(1).transpose(1, 2), mu.transpose(1, 2)).transpose(1, 2)
        o = O.align(logw, x_mask, mu, ls)
        assert torch.equal(o[0], yl) and o[2] == tp and torch.equal(o[4], attn) and torch.equal(o[5], mu_y)
        out.update({f"ls{i}": np.float32(ls), f"w_ceil{i}": w_ceil, f"y_lengths{i}": yl,
                    f"t_pad{i}": np.int64(tp), f"attn{i}": attn, f"mu_y{i}": mu_y})
    print("  oracle vs reference G1: bit-exact OK")
    save("g1_durations", logw=logw, x_mask=x_mask, x_lengths=xl, mu=mu, **out)


def decoder_module(c_cond):
    return ref_model.Decoder(in_channels=c_cond, out_channels=80, **{k: v for k, v in DEC.items()})


def g2_g3():
    for c_cond, tag in [(160, "lj"), (224, "vctk")]:
        dec = decoder_module(c_cond)
        sd = load_synth(dec, SEED + c_cond)
        rs = np.random.RandomState(c_cond)
        B, T = 2, 64
        yl = torch.tensor([64, 53])
        mask = O.sequence_mask(yl, T).unsqueeze(1).float()
        x = torch.from_numpy(rs.standard_normal((B, 80, T)).astype(np.float32))
        mu = torch.from_numpy(rs.standard_normal((B, 80, T)).astype(np.float32)) * mask
        spks = torch.from_numpy(rs.standard_normal((B, 64)).astype(np.float32)) if c_cond == 224 else None
        # per-block intermediates via forward hooks
        inter = {}
        hooks = [
            dec.down_blocks[0][0].register_forward_hook(lambda m, i, o: inter.__setitem__("down0_res", o)),
            dec.down_blocks[0][1][0].register_forward_hook(lambda m, i, o: inter.__setitem__("down0_tb", o)),
            dec.mid_blocks[1][1][0].register_forward_hook(lambda m, i, o: inter.__setitem__("mid1_tb", o)),
            dec.up_blocks[0][2].register_forward_hook(lambda m, i, o: inter.__setitem__("up0_out", o)),
            dec.up_blocks[1][1][0].register_forward_hook(lambda m, i, o: inter.__setitem__("up1_tb", o)),
        ]
        res = {}
        with torch.no_grad():
            for ti, tval in enumerate([0.0, 0.5]):
                t = torch.tensor([tval] * B)
                out = dec(x, mask, mu, t, spks)
                res[f"out_t{ti}"] = out
                res[f"t{ti}"] = np.float32(tval)
                if ti == 0:
                    for k, v in inter.items():
                        res[k] = v.clone()
                o = O.decoder_forward(sd, x, mask, mu, t, spks)
                close(o, out, 2e-5, f"G2[{tag}] decoder t={tval}")
        for h in hooks:
            h.remove()
        save(f"g2_decoder_{tag}", x=x, mask=mask, mu=mu, y_lengths=yl,
             spks=(spks if spks is not None else np.zeros((0,), np.float32)),
             manifest=np.array(manifest(dec)), seed=np.int64(SEED + c_cond), **res)

        # G3: CFM with injected z
        cfm_out = {}
        for solver, n in [("euler", 4), ("midpoint", 2)]:
            cfm = ref_model.CFM(n_feats=80, cfm_params={"solver": solver, "sigma_min": 1e-4},
                                n_spks=1, spk_emb_dim=64, estimator=dec)
            z0 = torch.from_numpy(np.random.RandomState(77).standard_normal((B, 80, T)).astype(np.float32))
            temp = 0.667
            orig = torch.randn_like
            torch.randn_like = lambda t, *a, **k: z0.clone()
            try:
                zT = cfm(mu, mask, n, temperature=temp, spks=spks)
            finally:
                torch.randn_like = orig
            o = O.cfm_solve(sd, mu, mask, n, z0 * temp, spks, solver)
            close(o, zT, 5e-5, f"G3[{tag}] cfm {solver} n={n}")
            cfm_out[f"z0_{solver}"] = z0
            cfm_out[f"zT_{solver}"] = zT
            cfm_out[f"n_{solver}"] = np.int64(n)
        save(f"g3_cfm_{tag}", mu=mu, mask=mask, spks=(spks if spks is not None else np.zeros((0,), np.float32)),
             temperature=np.float32(0.667), manifest=np.array(manifest(dec)), seed=np.int64(SEED + c_cond),
             **cfm_out)


def g4_g5():
    h = AttrDict(ref_v1)
    gen = ref_hifi.Generator(h)
    raw = load_synth(gen, SEED + 7)
    man = manifest(gen)
    gen.remove_weight_norm()
    folded_ref = {k: v.detach().clone() for k, v in gen.state_dict().items()}
    folded_or = O.fold_generator(raw)
    for k in ["conv_pre.weight", "ups.0.weight", "resblocks.4.convs1.1.weight", "conv_post.weight"]:
        close(folded_or[k], folded_ref[k], 1e-6, f"G4 fold {k}")
    rs = np.random.RandomState(5)
    B, T = 2, 16
    mel = torch.from_numpy((rs.standard_normal((B, 80, T)) * 2.0 - 5.5).astype(np.float32))
    stages = {}
    hooks = [gen.ups[i].register_forward_hook(lambda m, i_, o, i=i: stages.__setitem__(f"ups{i}", o))
             for i in range(4)]
    with torch.no_grad():
        wav = gen(mel)
    for hk in hooks:
        hk.remove()
    o = O.generator_forward(folded_ref, mel, dict(h))
    close(o, wav, 2e-6, "G4 generator")
    print(f"  wav stats: max|w|={wav.abs().max():.3f} std={wav.std():.3f}")
    # folded-weight slices (first 4 rows along dim 0) pin remove_weight_norm
    fold_check = {f"fold_{k.replace('.', '_')}": folded_ref[k][:4].clone() for k in
                  ["conv_pre.weight", "ups.0.weight", "resblocks.4.convs1.1.weight"]}
    save("g4_hifigan", mel=mel, wav=wav, manifest=np.array(man), seed=np.int64(SEED + 7),
         ups0=stages["ups0"], ups2=stages["ups2"][:, :, :512].clone(), **fold_check)

    # G5 denoiser (mode zeros) on the G4 audio (as main/notebook: [B, L])
    den = RefDenoiser(gen, mode="zeros")
    audio = wav.squeeze(1)
    with torch.inference_mode():
        out = den(audio, strength=0.00025)
        out_strong = den(audio, strength=0.05)
    bs = O.denoiser_bias_spec(folded_ref, dict(h))
    close(bs, den.bias_spec, 1e-6, "G5 bias_spec")
    close(O.denoise(audio, bs, 0.00025), out, 1e-6, "G5 denoise")
    close(O.denoise(audio, bs, 0.05), out_strong, 1e-6, "G5 denoise strong")
    save("g5_denoiser", audio=audio, bias_spec=den.bias_spec, out=out, out_strong=out_strong,
         strength=np.float32(0.00025), strength_strong=np.float32(0.05))


def g6():
    for n_spks, tag in [(1, "lj"), (109, "vctk")]:
        m = make_matcha(n_spks)
        sd = load_synth(m, SEED + 99 + n_spks)
        # shorten durations: every token gets ceil(exp(0.3)) = 2 frames, plus jitter from
        # a small random proj weight so lengths are ragged
        rs = np.random.RandomState(3)
        with torch.no_grad():
            m.encoder.proj_w.proj.weight.mul_(0.05)
            m.encoder.proj_w.proj.bias.fill_(0.3)
        sd["encoder.proj_w.proj.weight"] = m.encoder.proj_w.proj.weight.detach().clone()
        sd["encoder.proj_w.proj.bias"] = m.encoder.proj_w.proj.bias.detach().clone()
        B, Tx = 2, 23
        xl = torch.tensor([23, 15])
        x = torch.from_numpy(rs.randint(1, 178, size=(B, Tx))).long()
        x[:, 0::2] = 0
        x[1, 15:] = 0
        spk_emb = torch.from_numpy(rs.standard_normal((B, 64)).astype(np.float32)) if n_spks > 1 else None
        zs = {}

        def fake_randn(t, *a, **k):
            g = torch.Generator().manual_seed(4242)
            zs["z"] = torch.randn(t.shape, generator=g, dtype=t.dtype)
            return zs["z"].clone()

        orig = torch.randn_like
        torch.randn_like = fake_randn
        try:
            mel, yl, attn = m.synthesize(x, xl, n_timesteps=4, temperature=0.667, spks=spk_emb,
                                         length_scale=1.0)
        finally:
            torch.randn_like = orig
        hp = dict(n_channels=192, n_layers=6, n_heads=2, kernel_size=3, dp_kernel_size=3,
                  n_spks=n_spks)
        mo, ylo, ao = O.synthesize(sd, x, xl, 4, lambda mu: zs["z"] * 0.667, hp, spk_emb)
        assert torch.equal(ylo, yl) and torch.equal(ao, attn)
        close(mo, mel, 1e-4, f"G6[{tag}] synthesize mel")
        extra = {}
        with torch.no_grad():
            mu, logw, x_mask = m.encoder(x, xl, spk_emb)
            extra = dict(enc_mu=mu, enc_logw=logw, enc_x_mask=x_mask)
            mo2, lo2, xm2 = O.text_encoder(O.sub(sd, "encoder"), x, xl, hp, spk_emb)
            close(mo2, mu, 1e-5, f"G6[{tag}] encoder mu")
            close(lo2, logw, 1e-5, f"G6[{tag}] encoder logw")
        save(f"g6_synth_{tag}", x=x, x_lengths=xl, z=zs["z"], temperature=np.float32(0.667),
             n_timesteps=np.int64(4), mel=mel, y_lengths=yl, attn=attn,
             spks=(spk_emb if spk_emb is not None else np.zeros((0,), np.float32)),
             manifest=np.array(manifest(m)), seed=np.int64(SEED + 99 + n_spks),
             proj_w_weight=sd["encoder.proj_w.proj.weight"], proj_w_bias=sd["encoder.proj_w.proj.bias"],
             **extra)


if __name__ == "__main__":
    print("G1"); g1()
    print("G2/G3"); g2_g3()
    print("G4/G5"); g4_g5()
    print("G6"); g6()
