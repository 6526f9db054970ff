"""In-process A/B of the bf16 CFM solve (10 Euler steps, the bench's uniform-attention shapes) with the decoder's
FeedForward fused (mt_ffn) or as the two mt_vconv GEMMs, interleaved; also checks the two outputs are equal.
Usage: python tools/ffn_ab.py [B] [T] [reps] [rounds]"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "matcha-tts_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from matcha_hip import _lib as L_  # noqa: E402

if os.environ.get("MT_LIB"):  # timing experiments: another build of the library
    L_.LIB_PATH = os.environ["MT_LIB"]
from matcha_hip import runtime as rt  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
T = int(sys.argv[2]) if len(sys.argv) > 2 else 728
REPS = int(sys.argv[3]) if len(sys.argv) > 3 else 10
ROUNDS = int(sys.argv[4]) if len(sys.argv) > 4 else 3
dev = torch.device("cuda", 0)
m, g, den, msd, gsd = bench.build_models(dev, "bf16", 1234)
est = m.decoder.estimator
eng = est.engine()
packed = est.packed(dev)
gen = torch.Generator().manual_seed(5)
mu = torch.randn(B, 80, T, generator=gen).to(dev)
z = torch.randn(B, 80, T, generator=gen).to(dev)
lens = torch.randint(T * 2 // 3, T - 4, (B,), generator=gen)
mask = (torch.arange(T)[None, :] < lens[:, None]).float()[:, None, :].to(dev)
ymax = int(lens.max())
lib = L_.lib()
rt.set_ffn_min_frames(int(os.environ.get("FFN_MIN", "0")))  # default here: every level fused (the library's: 32768)
ws = torch.empty(lib.mt_cfm_workspace_bytes(eng.h, B, T, 10, L_.SOLVER_EULER), dtype=torch.uint8, device=dev)
st = torch.cuda.current_stream(dev)


def solve(out):
    L_.check(lib.mt_cfm_solve_bounded(eng.h, packed.data_ptr(), L_.ptr(z), 0.667, L_.ptr(mu), L_.ptr(mask), None, B, T,
                                      ymax, 10, L_.SOLVER_EULER, L_.ptr(out), ws.data_ptr(), ws.numel(),
                                      ctypes.c_void_p(st.cuda_stream)), "solve")


MODES = (1, 3, 2, 0)  # mt_ffn serial, serial + frame-only prefetch, overlapped epilogues; the two mt_vconv launches
NAME = {1: "fused", 3: "fused+pfb", 2: "fused+overlap", 0: "two-launch"}
outs = {k: torch.empty_like(mu) for k in MODES}
res = {k: [] for k in MODES}
for r in range(ROUNDS):
    for fused in MODES:
        rt.set_ffn(fused)
        for _ in range(2):
            solve(outs[fused])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(REPS):
            solve(outs[fused])
        torch.cuda.synchronize()
        res[fused].append((time.perf_counter() - t0) / REPS * 1e3)
rt.set_ffn(1)
for fused in MODES:
    v = sorted(res[fused])
    print(f"{NAME[fused]}: median {v[len(v) // 2]:.3f} ms per solve (B={B}, T={T}; {[round(x, 3) for x in v]})", flush=True)
for k in (1, 3, 2):
    print(f"{NAME[k]} vs two-launch bit-identical: {torch.equal(outs[k], outs[0])}, "
          f"max |diff| {(outs[k] - outs[0]).abs().max().item():.3e}")
