#!/usr/bin/env python3
"""Per-launch times of the vocoder's fused-pair / per-layer ResBlock launches (launch probe, PROBE_VCONV) at one
batch shape, grouped by kernel kind and kernel size k (from the probe's FLOP count), after a warm-up call.
Env knobs are read by the library (e.g. MT_VPAIR3); PAIR sets the vocoder pair mode. Usage: python tools/pair_probe.py [B] [T] [reps]"""
import os
import sys
from collections import defaultdict

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "matcha-tts_amd"))
import torch  # noqa: E402

from hifigan.config import v1  # noqa: E402
from hifigan.env import AttrDict  # noqa: E402
from hifigan.models import Generator  # noqa: E402
from matcha_hip import runtime as rt, synthetic  # noqa: E402
if os.environ.get("MT_LIB"):  # timing experiments: another build of the library
    import matcha_hip._lib as _L  # noqa: E402
    _L.LIB_PATH = os.environ["MT_LIB"]

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
T = int(sys.argv[2]) if len(sys.argv) > 2 else 728
R = int(sys.argv[3]) if len(sys.argv) > 3 else 3
g = Generator(AttrDict(v1), precision="bf16")
sd = synthetic.make_state_dict([(k, tuple(v.shape)) for k, v in g.state_dict().items()], 7)
g.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
g = g.cuda().eval()
g.remove_weight_norm()
if os.environ.get("PAIR"):  # vocoder pair mode (mt_vocoder_set_pair)
    g.engine().set_pair(int(os.environ["PAIR"]))
mel = (torch.randn(B, 80, T) * 2 - 5).cuda()
g(mel)
torch.cuda.synchronize()
acc = defaultdict(list)
for _ in range(R):
    rt.probe_start(rt.PROBE_VCONV, 128)
    g(mel)
    det = rt.probe_detail()
    rt.probe_stop()
    for d in det:
        # C and samples per mel frame by kind; k from FLOPs = (2 convs if pair) * 2 * C^2 * k * B * L
        C, rate = {"vpair128": (128, 64), "vpair": (64, 128), "vpair32": (32, 256)}.get(d["kind"], (0, 0))
        k = round(d["flops"] / (2 * 2 * C * C * B * T * rate)) if C else 0
        acc[(d["kind"], k)].append(d["ms"])
tag = os.environ.get("MT_VPAIR3", "default") + " PAIR=" + os.environ.get("PAIR", "1") + " LIB=" + os.environ.get("MT_LIB", "-")
for key in sorted(acc):
    v = acc[key]
    print(f"[MT_VPAIR3={tag}] {key[0]:9s} k={key[1]:2d}: {len(v) // R} launches, mean {sum(v) / len(v):.3f} ms, "
          f"total {sum(v) / R:.3f} ms per call", flush=True)
