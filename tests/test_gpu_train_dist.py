"""The DDP training step for real: two ranks, both on cuda:0, over gloo (world 2), running the actual
MatchaTrainer / MatchaLightningModule step (train_standalone.py:623-707 under Lightning DDP, :863-874).

Checked:
  * start-up: rank 1 is built from DIFFERENT weights and after construction holds rank 0's bitwise (DDP's
    broadcast at wrap time); the module's mel_mean / mel_std are rank 0's after a forward (broadcast_buffers);
  * the all-reduced gradient is exactly the sum of the two ranks' local gradients (each computed by a world-1
    trainer on the same weights), and each local gradient matches autograd through the oracle on that rank's batch
    (relative L2 2e-3 over the flat gradient, as tests/test_gpu_train.py);
  * the update: the ranks are bitwise equal after optimizer_step, and equal (max |dp| 5e-7) to torch's
    clip_grad_norm_(5.0) + Adam(lr 1e-4) applied to the MEAN of the two ranks' gradients;
  * the logged losses are the mean over the ranks (self.log(..., sync_dist=True)).
Both ranks share one GPU here (the 8-GPU run uses one rank per GPU over RCCL); gloo moves the same bytes.
"""
import os
import socket
import sys

import pytest
import torch

from conftest import HP, PKG, REPO

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    for p in (PKG, REPO, os.path.join(REPO, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from test_gpu_train import _setup
        from matcha_hip.train import MatchaTrainer
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        sd0, _, _, _, _, _, _ = _setup(seed=26)
        sd = {k: (v + 0.01 if rank == 1 and torch.is_floating_point(v) else v) for k, v in sd0.items()}
        _, x, xl, y, yl, t, z = _setup(seed=30 + rank)
        own = [dist.new_group([r]) for r in range(world)][rank]  # a world-1 group per rank: local gradients
        tr = MatchaTrainer(sd, HP, dev, dropout=False)  # default group: world 2
        p0 = tr.params.flat.detach().cpu().clone()
        args = (x.to(dev), xl.to(dev), y.to(dev), yl.to(dev))
        out = tr.forward_backward(*args, t=t.to(dev), z=z.to(dev))
        g_sum = tr.grads.flat.detach().cpu().clone()
        loc = MatchaTrainer({k: sd0[k] for k in sd0}, HP, dev, dropout=False, process_group=own)
        loc.forward_backward(*args, t=t.to(dev), z=z.to(dev))
        g_loc = loc.grads.flat.detach().cpu().clone()
        tr.optimizer_step()
        torch.cuda.synchronize()
        res = {"p0": p0, "g_sum": g_sum, "g_loc": g_loc, "p1": tr.params.flat.detach().cpu().clone(),
               "names": list(tr.grads.names), "loss": float(out["loss"])}
        # the Lightning drop-in under DDP: buffers, synced logging, rank-equal update
        from types import SimpleNamespace

        import train_standalone as TS
        from conftest import DEC, DP, ENC
        mod = TS.MatchaLightningModule(178, 1, 64, SimpleNamespace(**ENC), SimpleNamespace(**DEC),
                                       {"solver": "euler", "sigma_min": 1e-4}, SimpleNamespace(**DP),
                                       {"mel_mean": 0.0, "mel_std": 1.0})
        mod.model.load_state_dict(sd)
        mod.to(dev)
        opt = mod.configure_optimizers()
        torch.manual_seed(7 + rank)
        batch = {"x": args[0], "x_lengths": args[1], "y": args[2], "y_lengths": args[3]}
        loss = mod.training_step(batch, 0)
        opt.step()
        torch.cuda.synchronize()
        res.update(mod_loss=loss.detach().cpu().clone(), mod_logged=mod.logged["train/loss"].detach().cpu().clone(),
                   mel=(float(mod.mel_mean), float(mod.mel_std)),
                   mod_p=torch.cat([v.detach().reshape(-1).cpu() for v in mod.model.state_dict().values()
                                    if torch.is_floating_point(v)]))
        # by value (numpy): a worker's shared-memory tensors die with it
        q.put((rank, {k: (v.numpy() if isinstance(v, torch.Tensor) else v) for k, v in res.items()}))
    except Exception as e:  # surface the error in the parent
        import traceback
        q.put((rank, {"error": traceback.format_exc()}))
    finally:
        dist.destroy_process_group()


def test_ddp_world2_step_on_one_gpu():
    import torch.multiprocessing as mp
    from test_gpu_train import _oracle_grads, _setup
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert "error" not in res[r], res[r].get("error")
        res[r] = {k: (torch.from_numpy(v) if hasattr(v, "dtype") and hasattr(v, "shape") else v)
                  for k, v in res[r].items()}
    r0, r1 = res[0], res[1]
    # DDP start-up: rank 1 (built from other weights) holds rank 0's
    assert torch.equal(r0["p0"], r1["p0"])
    # gradient all-reduce = the exact sum of the local gradients
    assert torch.equal(r0["g_sum"], r1["g_sum"])
    assert torch.equal(r0["g_sum"], r0["g_loc"] + r1["g_loc"])
    # each local gradient vs autograd through the oracle on that rank's batch
    sd0, _, _, _, _, _, _ = _setup(seed=26)
    mean_ref = None
    for r in range(world):
        _, x, xl, y, yl, t, z = _setup(seed=30 + r)
        _, g = _oracle_grads(sd0, x, xl, y, yl, t, z)
        flat = torch.cat([g[n].reshape(-1) for n in r0["names"]])
        err = float((res[r]["g_loc"].double() - flat.double()).norm() / flat.double().norm())
        assert err < 2e-3, (r, err)
        mean_ref = flat / world if mean_ref is None else mean_ref + flat / world
    # the update: ranks bitwise equal; torch clip + Adam on the mean gradient
    assert torch.equal(r0["p1"], r1["p1"])
    p = r0["p0"].clone().requires_grad_(True)
    p.grad = (r0["g_sum"] / world).clone()
    torch.nn.utils.clip_grad_norm_([p], 5.0)
    opt = torch.optim.Adam([p], lr=1e-4)
    opt.step()
    assert (r0["p1"] - p.detach()).abs().max().item() < 5e-7
    # Lightning drop-in: rank 0's buffers everywhere, logged loss = mean over ranks, rank-equal weights
    # (the model's state dict carries mel_mean / mel_std: rank 1 loaded them +0.01, rank 0's values win)
    assert r0["mel"] == r1["mel"] == (float(sd0["mel_mean"]), float(sd0["mel_std"]))
    assert torch.equal(r0["mod_logged"], r1["mod_logged"])
    assert torch.equal(r0["mod_logged"], (r0["mod_loss"] + r1["mod_loss"]) / world)
    assert torch.equal(r0["mod_p"], r1["mod_p"])
    print(f"world-2 DDP step: grad mean vs oracle ok, losses {r0['loss']:.4f} / {r1['loss']:.4f}, "
          f"logged mean {float(r0['mod_logged']):.4f}")
