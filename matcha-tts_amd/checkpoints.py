"""On-disk formats (§8f rank 4): the two checkpoint layouts the reference's inference script loads.

- Matcha (main.py:93-121): a Lightning `.ckpt` whose `state_dict` keys carry the LightningModule's
  `model.` prefix (train_standalone.py:618-621 registers `mel_mean` / `mel_std` on the LightningModule
  AND assigns them to `model`, so both `mel_mean` and `model.mel_mean` appear), or a bare state dict.
  The prefix is stripped key by key in file order, later keys overwriting earlier ones, exactly as
  main.py:104-111 does; `load_state_dict` then runs strict.
- HiFi-GAN (main.py:142-150): `{"generator": state_dict}` with weight-norm `weight_g` / `weight_v`
  keys, loaded into the Generator before `remove_weight_norm()`.

Files are read ONLY with `torch.load(weights_only=True)` (tensors, containers and primitives; nothing
in the file is executed). A Lightning checkpoint that pickles other objects (callback or
hyper-parameter classes) is refused by that loader; name those classes in `safe_globals` to allowlist
them (torch.serialization.safe_globals) — there is deliberately no `weights_only=False` path.
"""
from typing import Dict, Iterable, Optional

import torch


def _load(path_or_obj, map_location, safe_globals: Optional[Iterable] = None):
    if isinstance(path_or_obj, dict):
        return path_or_obj
    allow = list(safe_globals or [])
    with torch.serialization.safe_globals(allow):
        return torch.load(path_or_obj, map_location=map_location, weights_only=True)


def matcha_state_dict(ckpt) -> Dict[str, torch.Tensor]:
    """main.py:96-111: the checkpoint's state dict with the `model.` prefix stripped."""
    state = ckpt["state_dict"] if "state_dict" in ckpt else ckpt
    out = {}
    for k, v in state.items():
        out[k[6:] if k.startswith("model.") else k] = v
    return out


def load_matcha(model: torch.nn.Module, path_or_obj, map_location="cpu", safe_globals: Optional[Iterable] = None):
    """Load a Matcha Lightning checkpoint (or bare state dict) into `model` (strict), return the model."""
    model.load_state_dict(matcha_state_dict(_load(path_or_obj, map_location, safe_globals)))
    return model


def load_hifigan(generator: torch.nn.Module, path_or_obj, map_location="cpu",
                 safe_globals: Optional[Iterable] = None, remove_weight_norm: bool = True):
    """main.py:146-149: state["generator"] into the Generator, then fold weight norm (as main.py does)."""
    state = _load(path_or_obj, map_location, safe_globals)
    generator.load_state_dict(state["generator"] if "generator" in state else state)
    if remove_weight_norm:
        generator.remove_weight_norm()
    return generator
