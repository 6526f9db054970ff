"""Multi-rank bench logic on CPU (gloo, world_size 2): utterance shards are disjoint slices of one
global synthetic set (weak scaling, no data-path collective), and the job time / work reduction is
MAX over ranks of the timed region and SUM of useful frames."""
import os
import socket
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "matcha-tts_amd"))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    x, xl = bench.shard_inputs(rank, world, 4, 1234)
    el, fr = bench.reduce_over_ranks(1.0 + rank, 100 * (rank + 1), dist, torch.device("cpu"))
    q.put((rank, x.numpy(), xl.numpy(), el, fr))
    dist.barrier()
    dist.destroy_process_group()


def test_bench_sharding_and_reduction_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from matcha_hip import synthetic
    gx, gl = synthetic.synthetic_text(4 * world, seed=1234)
    for rank, x, xl, el, fr in res:
        assert el == 2.0 and fr == 300  # max of (1, 2); sum of (100, 200)
        assert np.array_equal(xl, gl[rank * 4:(rank + 1) * 4])
        assert x.shape[1] == xl.max()
        assert np.array_equal(x, gx[rank * 4:(rank + 1) * 4, : x.shape[1]])
    # shards are disjoint slices: together they are the global set
    assert np.array_equal(np.concatenate([r[2] for r in res]), gl)


def _run_bench(args, env_extra=None, timeout=180):
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=timeout)


def test_bench_gpus_flag_launches_its_own_ranks():
    """``python bench.py --gpus 2`` with no launcher in the environment starts 2 rank processes itself (RANK /
    WORLD_SIZE / MASTER_* set per child, torch.distributed.run style), and rank 0 prints ONE line with n_gpus 2 and
    the SUM of both shards' frames (CPU rehearsal: gloo ranks, host stand-in for the step)."""
    import json

    from matcha_hip import synthetic
    r = _run_bench(["--gpus", "2", "--steps", "3", "--warmup", "0", "--batch", "4", "--cpu-selftest"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    _, gl = synthetic.synthetic_text(8, seed=1234)
    assert out["n_gpus"] == 2 and out["steps"] == 3 and out["frames_per_step"] == int(gl.sum()) * 3


def test_bench_rejects_world_mismatch():
    """--gpus must match the world a launcher started: WORLD_SIZE=1 with --gpus 2 exits non-zero instead of
    measuring one GPU and labelling it two"""
    r = _run_bench(["--gpus", "2", "--steps", "1", "--cpu-selftest"], {"WORLD_SIZE": "1", "RANK": "0",
                                                                         "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr
