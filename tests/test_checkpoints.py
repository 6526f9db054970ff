"""§8f rank 4 on-disk formats (CPU): Lightning-style Matcha checkpoints (model. prefix, duplicate
mel statistics keys) and HiFi-GAN {"generator": ...} files round-trip into the drop-in modules through
checkpoints.py, read with torch.load(weights_only=True)."""
import torch

import checkpoints
from conftest import make_generator, make_matcha


def test_matcha_lightning_checkpoint(tmp_path):
    src = make_matcha(1, "fp32")
    with torch.no_grad():
        for i, p in enumerate(src.parameters()):
            p.copy_(torch.full_like(p, 0.001 * (i % 97)))
        src.mel_mean.fill_(-5.5366)
        src.mel_std.fill_(2.1161)
    sd = src.state_dict()
    lightning = {"mel_mean": torch.tensor(123.0), "mel_std": torch.tensor(7.0)}  # LightningModule's own buffers
    lightning.update({"model." + k: v for k, v in sd.items()})                    # then model.* (file order)
    path = tmp_path / "last.ckpt"
    torch.save({"epoch": 3, "global_step": 1000, "state_dict": lightning}, path)
    dst = checkpoints.load_matcha(make_matcha(1, "fp32"), path)
    for k, v in sd.items():
        assert torch.equal(dst.state_dict()[k], v), k
    # bare state dict, no prefix
    dst2 = checkpoints.load_matcha(make_matcha(1, "fp32"), dict(sd))
    assert torch.equal(dst2.mel_std, sd["mel_std"])


def test_hifigan_generator_file(tmp_path):
    src = make_generator("fp32")
    torch.save({"generator": src.state_dict()}, tmp_path / "g_02500000")
    dst = checkpoints.load_hifigan(make_generator("fp32"), tmp_path / "g_02500000", remove_weight_norm=False)
    for k, v in src.state_dict().items():
        assert torch.equal(dst.state_dict()[k], v), k
    folded = checkpoints.load_hifigan(make_generator("fp32"), tmp_path / "g_02500000")
    assert not any(k.endswith("weight_g") for k in folded.state_dict())


class _HParams:  # stands in for a pickled Lightning hyper-parameter object
    def __init__(self, lr):
        self.lr = lr


def test_pickled_objects_need_an_allowlist(tmp_path):
    """Only weights_only=True loading exists: a pickled non-tensor object is refused unless its class
    is allowlisted (safe_globals); nothing in the file is ever executed."""
    import pickle

    import pytest
    sd = make_matcha(1, "fp32").state_dict()
    path = tmp_path / "with_hparams.ckpt"
    torch.save({"hyper_parameters": _HParams(1e-4), "state_dict": {"model." + k: v for k, v in sd.items()}}, path)
    with pytest.raises(pickle.UnpicklingError):
        checkpoints.load_matcha(make_matcha(1, "fp32"), path)
    dst = checkpoints.load_matcha(make_matcha(1, "fp32"), path, safe_globals=[_HParams])
    assert torch.equal(dst.state_dict()["mel_std"], sd["mel_std"])
