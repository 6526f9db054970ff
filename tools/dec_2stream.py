"""A/B: the 10-step CFM solve of the bench batch (B=32, T=728) as one solve vs two half-batch solves on two
streams (separate workspaces), to see whether the decoder's per-launch ramp / tail time overlaps.
Usage: python tools/dec_2stream.py [B] [T] [reps]"""
import ctypes
import sys
import time

import os as _os

_ROOT = _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))
sys.path.insert(0, _ROOT)
sys.path.insert(0, _os.path.join(_ROOT, "matcha-tts_amd"))

import torch

import bench
from matcha_hip import _lib as rt
from matcha_hip._lib import lib

if __import__("os").environ.get("MT_LIB"):  # timing experiments: another build of the library
    rt.LIB_PATH = __import__("os").environ["MT_LIB"]

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
T = int(sys.argv[2]) if len(sys.argv) > 2 else 728
REPS = int(sys.argv[3]) if len(sys.argv) > 3 else 10
dev = torch.device("cuda", 0)
m, g, den, msd, gsd = bench.build_models(dev, "bf16", 1234)
est = m.decoder.estimator
eng = est.engine()
packed = est.packed(dev)
gen = torch.Generator().manual_seed(5)
mu = (torch.randn(B, 80, T, generator=gen)).to(dev)
z = torch.randn(B, 80, T, generator=gen).to(dev)
lens = torch.randint(T * 2 // 3, T - 4, (B,), generator=gen)
mask = (torch.arange(T)[None, :] < lens[:, None]).float()[:, None, :].to(dev)
ymax = int(lens.max())
L = lib()


def solve(b0, b1, out, ws, st):
    nb = b1 - b0
    rt.check(L.mt_cfm_solve_bounded(eng.h, packed.data_ptr(), rt.ptr(z[b0:b1]), 0.667, rt.ptr(mu[b0:b1]),
                                    rt.ptr(mask[b0:b1]), None, nb, T, ymax, 10, rt.SOLVER_EULER,
                                    rt.ptr(out[b0:b1]), ws.data_ptr(), ws.numel(), ctypes.c_void_p(st.cuda_stream)),
             "solve")


out1 = torch.empty_like(mu)
out2 = torch.empty_like(mu)
wsf = torch.empty(L.mt_cfm_workspace_bytes(eng.h, B, T, 10, rt.SOLVER_EULER), dtype=torch.uint8, device=dev)
h = B // 2
wsa = torch.empty(L.mt_cfm_workspace_bytes(eng.h, h, T, 10, rt.SOLVER_EULER), dtype=torch.uint8, device=dev)
wsb = torch.empty(L.mt_cfm_workspace_bytes(eng.h, B - h, T, 10, rt.SOLVER_EULER), dtype=torch.uint8, device=dev)
s0 = torch.cuda.current_stream(dev)
s1 = torch.cuda.Stream(dev)


def one():
    solve(0, B, out1, wsf, s0)


def two():
    s1.wait_stream(s0)
    solve(0, h, out2, wsa, s0)
    solve(h, B, out2, wsb, s1)
    s0.wait_stream(s1)


for name, fn in (("one", one), ("two", two), ("one", one), ("two", two)):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(REPS):
        fn()
    torch.cuda.synchronize()
    print(f"{name}: {(time.perf_counter() - t0) / REPS * 1e3:.3f} ms per solve (B={B}, T={T})")
d = (out1 - out2).abs().max().item()
print(f"max |one - two| = {d:.3e}")
