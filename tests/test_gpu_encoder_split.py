"""The text encoder's split-bf16 FFN (encoder precision "fp32x3", mt_encoder_set_split; mt_vconv's VConvArgs::f32 == 2)
against the fp32 oracle (model.py:375-393, 452-535). Every fp32 FFN operand is stored as three bf16 parts and each
product summed from the six bf16 MFMA products whose parts reach 2^-16, in fp32: fp32-level arithmetic on the bf16
pipe. The bar is the exact-fp32 mode's: mu within 1e-4 (rel-RMS), logw within 1e-5 (max |d|), and on unforced
duration weights the index path (ceil(exp(logw)), y_lengths, the alignment; model.py:1273-1289) equal to the
oracle's at the bench's batches."""
import pytest
import torch

from conftest import make_matcha, rel_rms

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
SPLIT_TAG = 2 << 20  # launch-log flag of a split-mode mt_vconv launch (mt_vconv.hip launch_vconv_split)
HP = dict(n_channels=192, n_layers=6, n_heads=2, kernel_size=3, dp_kernel_size=3, n_spks=1)


@pytest.mark.parametrize("B", [32, 256])
def test_fp32x3_encoder_bench_batch_vs_oracle(B):
    import bench
    from matcha_hip import runtime as rt
    from oracle import matcha_oracle as O
    m, _, _, msd, _ = bench.build_models(DEV, "bf16", 1234)
    m.set_precision("bf16", encoder_precision="fp32x3")
    x, xl = bench.shard_inputs(0, 1, B, 1234)
    rt.vconv_log_start()
    with torch.inference_mode():
        mu, logw, xm = m.encoder(x.to(DEV), xl.to(DEV))
    torch.cuda.synchronize()
    log = rt.vconv_log_stop()
    # the FFN convs ran in the split mode: conv 1 (relu, mask, 6-plane output) and conv 2 (residual, mask), 6 layers
    split = [r for r in log if r["ef"] & SPLIT_TAG]
    assert len(split) == 12, len(split)
    assert {r["cin"] for r in split} == {6 * 192, 6 * 768}
    sd = {k[len("encoder."):]: v.cpu() for k, v in msd.items() if k.startswith("encoder.")}
    mu_o, logw_o, xm_o = O.text_encoder(sd, x, xl, HP)
    assert torch.equal(xm.cpu(), xm_o)
    e_mu = rel_rms(mu.cpu(), mu_o)
    e_logw = (logw.cpu() - logw_o).abs().max().item()
    print(f"encoder fp32x3 B={B} Tx={x.shape[1]}: mu rel-RMS {e_mu:.3e}, logw max|d| {e_logw:.2e}")
    assert e_mu < 1e-4 and e_logw <= 1e-5, (e_mu, e_logw)


@pytest.mark.parametrize("B", [32, 256])
def test_fp32x3_index_path_bit_exact_unforced_durations(B):
    """As test_gpu_parity_bf16.py::test_bf16_model_index_path_bit_exact_unforced_durations, with the split FFN: a real
    (not forced) duration head, logw within 1e-5 of the oracle's, and the durations / y_lengths / alignment equal."""
    from matcha_hip import runtime as rt
    from matcha_hip import synthetic
    from oracle import matcha_oracle as O
    m = make_matcha(1, precision="bf16")
    m.set_precision("bf16", encoder_precision="fp32x3")
    sd = {k: torch.from_numpy(v) for k, v in synthetic.make_state_dict(
        [(k, tuple(v.shape)) for k, v in m.state_dict().items()], 77).items()}
    assert float(sd["encoder.proj_w.proj.weight"].abs().sum()) > 0
    m.load_state_dict(sd)
    m = m.to(DEV).eval()
    x, xl = synthetic.synthetic_text(B, seed=1234)
    x, xl = torch.from_numpy(x)[:, : int(xl.max())].contiguous(), torch.from_numpy(xl)
    with torch.inference_mode():
        mu, logw, xm = m.encoder(x.to(DEV), xl.to(DEV))
        w_ceil, cum, yl = rt.durations(logw, xm, 1.0)
    esd = {k[len("encoder."):]: v for k, v in sd.items() if k.startswith("encoder.")}
    mu_o, logw_o, xm_o = O.text_encoder(esd, x, xl, HP)
    e_logw = (logw.cpu() - logw_o).abs().max().item()
    e_mu = rel_rms(mu.cpu(), mu_o)
    wc_o, yl_o = O.durations(logw_o, xm_o)
    print(f"fp32x3 unforced durations B={B}: logw max|d| {e_logw:.2e}, mu rel-RMS {e_mu:.2e}")
    assert torch.equal(xm.cpu(), xm_o)
    assert e_logw <= 1e-5 and e_mu < 1e-4, (e_logw, e_mu)
    assert torch.equal(yl.cpu(), yl_o), "y_lengths must be bit-exact"
    assert torch.equal(w_ceil.cpu(), wc_o)


def test_fp32x3_toggle_and_fp32_mode_unchanged():
    """set_split(0) on the same engine is the exact-fp32 path (its bits unchanged by the split images in the packed
    weights), and the split path is deterministic."""
    import bench
    m, _, _, _, _ = bench.build_models(DEV, "bf16", 99)
    x, xl = bench.shard_inputs(0, 1, 8, 99)
    outs = {}
    for prec in ("fp32", "fp32x3", "fp32x3"):
        m.set_precision("bf16", encoder_precision=prec)
        with torch.inference_mode():
            mu, logw, _ = m.encoder(x.to(DEV), xl.to(DEV))
        outs.setdefault(prec, []).append(mu.cpu())
    assert torch.equal(outs["fp32x3"][0], outs["fp32x3"][1])
    assert not torch.equal(outs["fp32x3"][0], outs["fp32"][0])  # the split path really ran
    assert rel_rms(outs["fp32x3"][0], outs["fp32"][0]) < 1e-5
