"""Golden vectors for Monotonic Alignment Search (§8f rank 3), produced by the reference's own
`maximum_path` (train_standalone.py:280-325).

train_standalone.py does not import here (torchaudio / lightning / numba are absent), so this script
parses the file with `ast`, compiles only the `maximum_path` function and runs it with
NUMBA_AVAILABLE = False (the reference's pure-Python branch). Run once in the build container:
    python tests/golden/make_golden_mas.py   ->  tests/golden/g7_mas.npz
"""
import ast
import os

import numpy as np
import torch

REF = "/root/reference/train_standalone.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "g7_mas.npz")


def reference_maximum_path():
    tree = ast.parse(open(REF).read())
    fn = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "maximum_path")
    ns = {"np": np, "torch": torch, "NUMBA_AVAILABLE": False}
    exec(compile(ast.Module(body=[fn], type_ignores=[]), REF, "exec"), ns)
    return ns["maximum_path"]


def case(rng, t_xs, t_ys, Tx, Ty, kind):
    B = len(t_xs)
    if kind == "normal":
        v = rng.standard_normal((B, Tx, Ty)).astype(np.float32)
    elif kind == "ties":  # small integers: many equal partial sums, exercises the strict '>'
        v = rng.integers(-2, 3, (B, Tx, Ty)).astype(np.float32)
    else:  # log-prior scale (train_standalone.py:638-644): large negative values
        v = (-0.5 * rng.standard_normal((B, Tx, Ty)) ** 2 * 80 - 73.5).astype(np.float32)
    xm = (np.arange(Tx)[None] < np.array(t_xs)[:, None]).astype(np.float32)
    ym = (np.arange(Ty)[None] < np.array(t_ys)[:, None]).astype(np.float32)
    mask = xm[:, :, None] * ym[:, None, :]
    return v, mask


def main():
    ref = reference_maximum_path()
    rng = np.random.default_rng(7)
    specs = [
        ([7, 5, 3], [20, 13, 3], 7, 20, "normal"),     # ragged, t_x == t_y edge
        ([6, 6], [15, 9], 6, 15, "ties"),
        ([1, 4], [5, 4], 4, 5, "normal"),               # one token; t_x == t_y
        ([33, 20], [120, 61], 33, 120, "logprior"),
        ([9], [6], 9, 6, "normal"),                     # t_x > t_y (columns with no visited cell)
    ]
    out = {}
    for i, (t_xs, t_ys, Tx, Ty, kind) in enumerate(specs):
        v, mask = case(rng, t_xs, t_ys, Tx, Ty, kind)
        p = ref(torch.from_numpy(v), torch.from_numpy(mask)).numpy()
        out[f"c{i}_neg"], out[f"c{i}_mask"], out[f"c{i}_path"] = v, mask, p
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, len(specs), "cases")


if __name__ == "__main__":
    main()
