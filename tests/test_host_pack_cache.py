"""Host logic of runtime.PackCache (CPU): a packed weight buffer is reused only while the module's state
tensors are unchanged (same tensors, addresses and version counters) and no parameter / buffer / module
registration happened since; `trust_next` skips exactly one check."""
import torch
from torch import nn

from matcha_hip import runtime as rt


def _mod():
    return nn.Sequential(nn.Linear(4, 3), nn.Linear(3, 2))


def test_hit_until_in_place_update():
    m = _mod()
    c = rt.PackCache()
    key = ("bf16", "cuda:0")
    assert c.get(key) is None
    c.put(key, list(m.state_dict(keep_vars=True).values()), "P1")
    assert c.get(key) == "P1"
    with torch.no_grad():
        m[0].weight.mul_(2.0)          # in-place update: version counter moves
    assert c.get(key) is None
    c.put(key, list(m.state_dict(keep_vars=True).values()), "P2")
    assert c.get(key) == "P2"
    m[1].weight.data = torch.zeros(2, 3)  # storage swap without a registration: address moves
    assert c.get(key) is None


def test_registration_invalidates():
    m = _mod()
    c = rt.PackCache()
    key = ("fp32", "cuda:0")
    c.put(key, list(m.state_dict(keep_vars=True).values()), "P")
    m[0].weight = nn.Parameter(torch.ones(3, 4))  # re-registration (e.g. remove_weight_norm)
    assert c.get(key) is None
    c.put(key, list(m.state_dict(keep_vars=True).values()), "P")
    m.register_buffer("extra", torch.zeros(1))
    assert c.get(key) is None


def test_trust_next_skips_one_check():
    m = _mod()
    c = rt.PackCache()
    key = ("bf16", "cuda:0")
    c.put(key, list(m.state_dict(keep_vars=True).values()), "P")
    c.trust_next(key)
    with torch.no_grad():
        m[0].bias.add_(1.0)
    assert c.get(key) == "P"   # trusted once
    assert c.get(key) is None  # then checked again
    c.trust_next(("other", "x"))  # unknown key: no effect
    assert not c.trusted
