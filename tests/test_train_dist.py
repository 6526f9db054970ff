"""Bucketed gradient all-reduce of the training step (matcha_hip.train.GradBuckets) on CPU with gloo,
world_size 2: buckets are issued while the backward is still marking gradients (overlap), the reduced
flat buffer is the SUM over ranks, and a gradient that is never produced or produced twice is an error.
The reference gets this from Lightning DDP (train_standalone.py:863-874)."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "matcha-tts_amd"))

SHAPES = [("a", (7,)), ("b", (3, 5)), ("c", (16,)), ("d", (2, 2, 2)), ("e", (33,)), ("f", (1,)), ("g", (40,))]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from matcha_hip.train import FlatBuffer, GradBuckets
    try:
        buf = FlatBuffer(SHAPES, "cpu")
        gb = GradBuckets(buf.spans, buf.flat, bucket_bytes=64)
        out = {"n_buckets": len(gb.ranges), "world": gb.world}
        for step in range(2):
            gb.reset()
            buf.flat.copy_(torch.arange(buf.flat.numel(), dtype=torch.float32) * (rank + 1) + step)
            issued_during = []
            for n, _ in SHAPES:
                gb.mark(n)
                issued_during.append(len(gb.handles))
            gb.finish()
            out[f"flat{step}"] = buf.flat.clone()
            out[f"issued{step}"] = issued_during
            out[f"order{step}"] = list(gb.issued)
        gb.reset()
        with pytest.raises(RuntimeError, match="twice"):
            gb.mark("a")
            gb.mark("a")
        gb.reset()
        for n, _ in SHAPES[:-1]:
            gb.mark(n)
        with pytest.raises(RuntimeError, match="no gradient"):
            gb.finish()
        q.put((rank, out))
    finally:
        # the incomplete last bucket was never issued on either rank: nothing is left in flight
        dist.barrier()
        dist.destroy_process_group()


def test_grad_buckets_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n = sum(int(torch.tensor(s).prod()) for _, s in SHAPES)
    for step in range(2):
        want = torch.arange(n, dtype=torch.float32) * 3 + 2 * step  # rank0 (x1) + rank1 (x2)
        for r in range(world):
            out = res[r]
            assert out["world"] == 2 and out["n_buckets"] > 2
            assert torch.equal(out[f"flat{step}"], want)
            # buckets went out while later gradients were still being marked
            issued = out[f"issued{step}"]
            assert issued[-2] >= 2 and issued[-1] == out["n_buckets"] and issued == sorted(issued)
            assert out[f"order{step}"] == list(range(out["n_buckets"]))


def test_grad_buckets_layout_single_process():
    sys.path.insert(0, os.path.join(ROOT, "matcha-tts_amd"))
    from matcha_hip.train import FlatBuffer, GradBuckets
    buf = FlatBuffer(SHAPES, "cpu")
    gb = GradBuckets(buf.spans, buf.flat, bucket_bytes=64)
    assert gb.world == 1
    # contiguous buckets covering the buffer exactly, each at least 64 bytes except possibly the last
    assert gb.ranges[0][0] == 0 and gb.ranges[-1][1] == buf.flat.numel()
    for (a, e), (a2, _) in zip(gb.ranges, gb.ranges[1:]):
        assert e == a2 and 4 * (e - a) >= 64
    # views alias the flat buffer in declaration order
    buf.view["b"].fill_(5.0)
    o = dict((n, (o, k)) for n, o, k in buf.spans)["b"]
    assert torch.all(buf.flat[o[0]:o[0] + o[1]] == 5.0)
    # marking in reverse order issues the last bucket first
    for n, _ in reversed(SHAPES):
        gb.mark(n)
    assert gb.issued[0] == len(gb.ranges) - 1
    gb.finish()
