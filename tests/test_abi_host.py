"""C-ABI library + host logic tests (CPU only: no kernel launches)."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from conftest import REPO, make_decoder, make_generator, make_matcha


def header_functions():
    src = open(os.path.join(REPO, "include", "matcha_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mtt?_\w+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    from matcha_hip import _lib
    L = _lib.lib()
    names = header_functions()
    assert len(names) >= 25
    for n in names:
        assert hasattr(L, n), n
    # the ctypes signature table mirrors the header exactly
    assert sorted(_lib.SIGNATURES) == names
    assert L.mt_abi_version() == 1


def test_library_is_production_build():
    from matcha_hip import _lib
    assert _lib.lib().mt_build_experiments() == 0  # no timing-experiment macro (VPAIR_EXP, RB_EXP, ...) built in


def test_loader_refuses_experiment_build(tmp_path, monkeypatch):
    """A library reporting an experiment build (mt_build_experiments() != 0: tools/exp_build.sh) is refused by the
    product loader, so smoke() / bench.py / the tests cannot run wrong-result kernels; the timing tools name such
    a library explicitly with MT_LIB. Checked on a stub library exporting the header's symbols."""
    import subprocess
    from matcha_hip import _lib
    names = header_functions()
    src = "".join(f"int {n}(void) {{ return {8 if n == 'mt_build_experiments' else 0}; }}\n" for n in names)
    (tmp_path / "stub.c").write_text(src)
    so = tmp_path / "libstub.so"
    subprocess.run(["gcc", "-shared", "-fPIC", "-w", str(tmp_path / "stub.c"), "-o", str(so)], check=True)
    monkeypatch.setattr(_lib, "LIB_PATH", str(so))
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.delenv("MT_LIB", raising=False)
    with pytest.raises(_lib.HipPathError, match="timing-experiment build"):
        _lib.lib()
    monkeypatch.setenv("MT_LIB", str(so))  # the timing tools' explicit override loads it
    assert _lib.lib().mt_build_experiments() == 8


def test_library_is_gfx950_code_object():
    from matcha_hip import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_decoder_param_list_matches_estimator_state_dict():
    from matcha_hip import runtime as rt
    for c_cond in (160, 224):
        for prec in ("fp32", "bf16"):
            eng = rt.DecoderEngine(c_cond, 2, 1, 2, prec)
            sd = make_decoder(c_cond).state_dict()
            names = [n for n, _ in eng.specs]
            assert "_sinus_freq" in names
            for n, shape in eng.specs:
                if n == "_sinus_freq":
                    assert shape == (c_cond // 2,)
                    continue
                assert tuple(sd[n].shape) == shape, n
            # every estimator tensor is consumed
            assert set(sd) == set(names) - {"_sinus_freq"}
            assert eng.packed_bytes > 10e6
            L = rt.lib()
            assert L.mt_cfm_workspace_bytes(eng.h, 32, 576, 10, 0) > L.mt_cfm_workspace_bytes(eng.h, 1, 576, 10, 0)


def test_vocoder_param_list_matches_folded_generator():
    from matcha_hip import runtime as rt
    g = make_generator()
    g.remove_weight_norm()
    sd = g.state_dict()
    eng = rt.VocoderEngine(dict(g.h), "bf16")
    assert {n for n, _ in eng.specs} == set(sd)
    for n, shape in eng.specs:
        assert tuple(sd[n].shape) == shape
    assert eng.hop == 256


def test_c_abi_errors_are_reported():
    from matcha_hip import runtime as rt
    from matcha_hip._lib import HipPathError
    with pytest.raises(HipPathError, match="c_cond"):
        rt.DecoderEngine(150, 2, 1, 2, "fp32")
    with pytest.raises(ValueError):
        rt.dtype_code("fp8")
    L = rt.lib()
    h = ctypes.c_void_p()
    rc = L.mt_vocoder_create(1, 1, (ctypes.c_int * 1)(8), (ctypes.c_int * 1)(15), 512, 1, (ctypes.c_int * 1)(3), 1,
                             (ctypes.c_int * 1)(1), 0, ctypes.byref(h))
    assert rc != 0 and b"multiple" in L.mt_last_error()


def test_hot_path_fails_loudly_on_cpu():
    """No CPU fallback: every HIP entry point refuses host tensors."""
    from matcha_hip._lib import HipPathError
    m = make_matcha(1)
    x = torch.randint(1, 178, (1, 11))
    with pytest.raises(HipPathError):
        m.synthesize(x, torch.tensor([11]), n_timesteps=2)
    g = make_generator()
    with pytest.raises(HipPathError):
        g(torch.zeros(1, 80, 8))
    dec = make_decoder(160)
    with pytest.raises(HipPathError):
        dec(torch.zeros(1, 80, 8), torch.ones(1, 1, 8), torch.zeros(1, 80, 8), torch.zeros(1))


def test_fix_len_and_sequence_mask():
    import model
    for n, e in [(1, 4), (4, 4), (5, 8), (575, 576), (576, 576), (757, 760)]:
        assert model.fix_len_compatibility(n) == e
    m = model.sequence_mask(torch.tensor([2, 0, 3]), 4)
    assert m.tolist() == [[True, True, False, False], [False] * 4, [True, True, True, False]]


def test_synthetic_recipe_is_deterministic():
    from matcha_hip import synthetic
    shapes = [("a.weight", (4, 3, 2)), ("a.bias", (4,)), ("n.weight", (4,)), ("ff.net.0.alpha", (5,))]
    a = synthetic.make_state_dict(shapes, 7)
    b = synthetic.make_state_dict(list(reversed(shapes)), 7)
    for k in a:
        assert np.array_equal(a[k], b[k])
    c = synthetic.make_state_dict(shapes, 8)
    assert not np.array_equal(a["a.weight"], c["a.weight"])
    lens = synthetic.ljspeech_lengths(1000)
    assert lens.min() >= 96 and lens.max() <= 868 and 520 < lens.mean() < 610
    x, xl = synthetic.synthetic_text(4)
    assert (x[:, 0::2][:, : min(xl) // 2] == 0).all() and (xl >= 150).all() and (xl <= 251).all()


def test_precision_switch():
    m = make_matcha(1)
    m.set_precision("bf16")
    # the text encoder / duration predictor stay fp32 in the bf16 mode: the index path is exact only on fp32 logw
    assert m.decoder.estimator.precision == "bf16" and m.encoder.precision == "fp32"
    m.set_precision("bf16", encoder_precision="bf16")
    assert m.encoder.precision == "bf16"
    assert make_matcha(1, precision="bf16").encoder.precision == "fp32"
    with pytest.raises(ValueError):
        m.set_precision("int8")


def test_ragged_batch_limit_matches_the_kernels():
    """Generator.forward splits a ragged batch into chunks of runtime.RAGGED_MAX_BATCH utterances: the limit the
    kernels' LDS tile tables have (mt_ragged.h RAG_MAXB)."""
    from matcha_hip import runtime as rt
    src = open(os.path.join(REPO, "matcha-tts_amd", "csrc", "mt_ragged.h")).read()
    m = re.search(r"constexpr int RAG_MAXB = (\d+);", src)
    assert m and int(m.group(1)) == rt.RAGGED_MAX_BATCH
