"""Decoder kernel variants (mt_decoder_set_kernels) against the launches they replace, bit for bit: bit 0 the final
projection + ODE update (final_proj of mish(GroupNorm(final_block conv)) * mask, then z += dt * v, model.py
Decoder.forward / flow_matching.py solve_euler) on proj_euler_kernel instead of the generic conv kernel. Same
operations in the same order, so every output must be EQUAL, not close. Checked end to end through the bench's
text->wav step, and through mt_cfm_solve with the Euler and midpoint solvers (the half step and the master-less
first evaluation) eagerly, on graph capture and on replay, with the query-independent and the general attention."""
import pytest
import torch

from conftest import make_decoder

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _models():
    import bench
    return bench.build_models(DEV, "bf16", 1234)


PROJ_TAG = 0x20000  # launch-log record of proj_euler_kernel (mt_conv.hip launch_proj_euler)


def _step(models, x, xl, mask, log=None):
    import bench
    from matcha_hip import runtime as rt
    m, g, den, _, _ = models
    prev = rt.set_decoder_kernels(mask)
    try:
        torch.manual_seed(7)  # the same CFM noise z for every run (synthesize draws it with torch.randn_like)
        if log is not None:
            rt.vconv_log_start(20000)
        with torch.inference_mode():
            mel, yl, wav = bench.step(m, g, den, x, xl, 10, True)
        torch.cuda.synchronize()
    finally:
        if log is not None:
            log.extend(rt.vconv_log_stop(20000))
        rt.set_decoder_kernels(prev)
    return mel.cpu(), yl.cpu(), wav.cpu()


@pytest.mark.parametrize("B", [6, 40])
def test_decoder_kernels_bit_identical_bench_step(B):
    import bench
    models = _models()
    x, xl = bench.shard_inputs(0, 1, B, 4321 + B)
    x, xl = x.to(DEV), xl.to(DEV)
    log0, log1 = [], []
    base = _step(models, x, xl, 0, log0)
    assert torch.isfinite(base[0]).all()
    # the first run of each selection captures the solve's graph, so its launches are logged: the dedicated kernel
    # ran once per ODE step with bit 0 on, never with it off (not the generic conv in both runs)
    assert sum(r["ef"] == PROJ_TAG for r in log0) == 0
    for i, mask in enumerate((1, 1)):
        got = _step(models, x, xl, mask, log1 if i == 0 else None)
        if i == 0:
            assert sum(r["ef"] == PROJ_TAG for r in log1) == 10, len(log1)
        assert torch.equal(got[1], base[1])
        assert torch.equal(got[0], base[0]), (mask, (got[0] - base[0]).abs().max())
        assert torch.equal(got[2], base[2]), mask


@pytest.mark.parametrize("solver", ["euler", "midpoint"])
def test_decoder_kernels_bit_identical_solve(solver):
    from matcha_hip import runtime as rt
    from matcha_hip import synthetic
    dec = make_decoder(160, "bf16")
    sd = {k: torch.from_numpy(v) for k, v in synthetic.make_state_dict(
        [(k, tuple(v.shape)) for k, v in dec.state_dict().items()], 29).items()}
    dec.load_state_dict(sd)
    dec = dec.to(DEV).eval()
    lens, T = [300, 251, 120, 64], 304
    B = len(lens)
    eng = dec.engine()
    g = torch.Generator().manual_seed(5)
    mask = (torch.arange(T)[None] < torch.tensor(lens)[:, None]).float()[:, None]
    mu = (torch.randn(B, 80, T, generator=g) * mask).to(DEV)
    z = (torch.randn(B, 80, T, generator=g) * 0.667).to(DEV)
    mask = mask.to(DEV)

    def run(kmask, graphs, mv):
        prev = rt.set_decoder_kernels(kmask)
        eng.set_graphs(graphs)
        try:
            out = eng.solve(dec.packed(DEV), z, 1.0, mu, mask, None, 4, solver=solver, max_valid=mv)
            torch.cuda.synchronize()
            return out.cpu()
        finally:
            rt.set_decoder_kernels(prev)
            eng.set_graphs(1)

    for mv in (max(lens), 0):  # the query-independent attention at both levels; the general attention
        base = run(0, 0, mv)
        assert torch.isfinite(base).all()
        for graphs in (0, 1, 1):  # eager, graph capture, graph replay
            got = run(1, graphs, mv)
            assert torch.equal(got, base), (mv, graphs, (got - base).abs().max())
