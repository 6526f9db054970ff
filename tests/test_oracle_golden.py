"""Pin the CPU oracle to golden vectors produced by the reference itself (CPU only).

G1 duration/index path is checked bit-exact; the floating-point paths within the
fp32 drift measured between two runs of the reference (~1e-6).
"""
import json

import numpy as np
import torch

from conftest import HP, golden, t, weights_from
from oracle import matcha_oracle as O


def test_g1_durations_bit_exact():
    g = golden("g1_durations")
    logw, x_mask, mu = t(g["logw"]), t(g["x_mask"]), t(g["mu"])
    for i in range(2):
        yl, ymax, tp, ymask, attn, mu_y = O.align(logw, x_mask, mu, float(g[f"ls{i}"]))
        assert torch.equal(yl, t(g[f"y_lengths{i}"]))
        assert tp == int(g[f"t_pad{i}"]) and tp % 4 == 0 and tp >= ymax
        assert torch.equal(attn, t(g[f"attn{i}"]))
        assert torch.equal(mu_y, t(g[f"mu_y{i}"]))
        w_ceil, _ = O.durations(logw, x_mask, float(g[f"ls{i}"]))
        assert torch.equal(w_ceil, t(g[f"w_ceil{i}"]))


def test_g1_path_is_one_hot_and_monotonic():
    g = golden("g1_durations")
    attn = t(g["attn0"])[:, 0]
    yl = t(g["y_lengths0"])
    for b in range(attn.shape[0]):
        cols = attn[b].sum(0)
        assert torch.all(cols[: yl[b]] == 1) and torch.all(cols[yl[b]:] == 0)
        tok = attn[b].argmax(0)[: yl[b]]
        assert torch.all(tok[1:] >= tok[:-1])


def _decoder_case(tag):
    g = golden(f"g2_decoder_{tag}")
    sd = weights_from(g)
    spks = t(g["spks"]) if g["spks"].size else None
    return g, sd, spks


def test_g2_decoder_forward_and_intermediates():
    for tag in ("lj", "vctk"):
        g, sd, spks = _decoder_case(tag)
        x, mask, mu = t(g["x"]), t(g["mask"]), t(g["mu"])
        for ti in range(2):
            tt = torch.full((x.shape[0],), float(g[f"t{ti}"]))
            taps = {}
            out = O.decoder_forward(sd, x, mask, mu, tt, spks, taps=taps)
            assert (out - t(g[f"out_t{ti}"])).abs().max() < 2e-5, tag
            if ti == 0:  # make_golden.py kept the hooks of the t0 evaluation
                for k in ("down0_res", "down0_tb", "mid1_tb", "up0_out", "up1_tb"):
                    ref = t(g[k])
                    got = taps[k].transpose(1, 2) if k.endswith("_tb") else taps[k]  # hooks saw b t c there
                    assert (got - ref).abs().max() < 2e-5, (tag, k)
        # the first resnet block alone
        temb = O.time_mlp(O.sub(sd, "time_mlp"), torch.zeros(x.shape[0]), sd["time_mlp.linear_1.weight"].shape[1])
        xin = torch.cat([x, mu] + ([spks.unsqueeze(-1).expand(-1, -1, x.shape[-1])] if spks is not None else []), 1)
        r = O.resnet1d(O.sub(sd, "down_blocks.0.0"), xin, mask, temb)
        assert (r - t(g["down0_res"])).abs().max() < 1e-5


def test_g3_cfm_euler_midpoint():
    for tag in ("lj", "vctk"):
        g = golden(f"g3_cfm_{tag}")
        sd = weights_from(g)
        spks = t(g["spks"]) if g["spks"].size else None
        mu, mask, temp = t(g["mu"]), t(g["mask"]), float(g["temperature"])
        for solver in ("euler", "midpoint"):
            z = O.cfm_solve(sd, mu, mask, int(g[f"n_{solver}"]), t(g[f"z0_{solver}"]) * temp, spks, solver)
            assert (z - t(g[f"zT_{solver}"])).abs().max() < 5e-5, (tag, solver)


def test_g4_generator_and_weight_norm_fold():
    g = golden("g4_hifigan")
    raw = weights_from(g)
    folded = O.fold_generator(raw)
    for k in ["conv_pre.weight", "ups.0.weight", "resblocks.4.convs1.1.weight"]:
        ref = t(g["fold_" + k.replace(".", "_")])
        assert (folded[k][:4] - ref).abs().max() < 1e-6, k
    from hifigan.config import v1 as V1
    wav = O.generator_forward(folded, t(g["mel"]), V1)
    assert (wav - t(g["wav"])).abs().max() < 1e-5
    assert wav.shape == (2, 1, 16 * 256)


def test_g5_denoiser():
    g = golden("g5_denoiser")
    audio, bias = t(g["audio"]), t(g["bias_spec"])
    out = O.denoise(audio, bias, float(g["strength"]))
    assert (out - t(g["out"])).abs().max() < 1e-6
    out2 = O.denoise(audio, bias, float(g["strength_strong"]))
    assert (out2 - t(g["out_strong"])).abs().max() < 1e-6
    assert out.shape[-1] == 256 * (audio.shape[-1] // 256)


def test_g6_synthesize_end_to_end():
    for tag in ("lj", "vctk"):
        g = golden(f"g6_synth_{tag}")
        sd = weights_from(g)
        sd["encoder.proj_w.proj.weight"] = t(g["proj_w_weight"])
        sd["encoder.proj_w.proj.bias"] = t(g["proj_w_bias"])
        spks = t(g["spks"]) if g["spks"].size else None
        hp = dict(HP, n_spks=1 if tag == "lj" else 109)
        z = t(g["z"])
        mel, yl, attn = O.synthesize(sd, t(g["x"]), t(g["x_lengths"]), int(g["n_timesteps"]),
                                     lambda mu: z * float(g["temperature"]), hp, spks)
        assert torch.equal(yl, t(g["y_lengths"]))
        assert torch.equal(attn, t(g["attn"]))
        assert (mel - t(g["mel"])).abs().max() < 1e-4


def test_manifests_match_product_modules():
    """The drop-in modules expose exactly the reference state_dict keys and shapes."""
    from conftest import make_decoder, make_generator, make_matcha
    cases = [("g6_synth_lj", make_matcha(1)), ("g6_synth_vctk", make_matcha(109)),
             ("g2_decoder_lj", make_decoder(160)), ("g2_decoder_vctk", make_decoder(224)),
             ("g4_hifigan", make_generator())]
    for name, mod in cases:
        man = {k: tuple(s) for k, s in json.loads(str(golden(name)["manifest"]))}
        mine = {k: tuple(v.shape) for k, v in mod.state_dict().items()}
        assert man == mine, name
