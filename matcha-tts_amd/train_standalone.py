"""Drop-in for the training surface of the reference's ``train_standalone.py`` (§8f rank 3): the helpers the
training step calls and ``MatchaLightningModule`` (train_standalone.py:580-707), running the CFM training step
on the MI355X through ``matcha_hip.train.MatchaTrainer`` (hand-written HIP forward + backward, RCCL bucketed
gradient all-reduce, fused clip + Adam).

Lightning is not installed in this image, so ``MatchaLightningModule`` is a plain ``torch.nn.Module`` with
the reference's methods and the semantics Lightning adds around them made explicit:

    module = MatchaLightningModule(n_vocab, n_spks, spk_emb_dim, encoder_params, decoder_params, cfm_params,
                                   duration_predictor_params, data_statistics, learning_rate=1e-4)
    module.to("cuda")
    opt = module.configure_optimizers()          # clip 5.0 (train_standalone.py:869) + Adam(lr)
    loss = module.training_step(batch, i)        # forward + backward (+ all-reduce on DDP ranks)
    opt.step(); opt.zero_grad()

``module.model`` is the drop-in ``model.MatchaTTS``; after ``opt.step()`` its parameters hold the trained
weights, so ``module.model.synthesize(...)`` (and ``state_dict()``) see the update. The data module, the
CLI and the Lightning Trainer loop (:714-900) are out of scope.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

import model as _model
from hifigan.meldataset import mel_spectrogram  # noqa: F401  (train_standalone.py:164-201, on the GPU)
from matcha_hip import runtime as rt
from matcha_hip.train import MatchaTrainer
from model import fix_len_compatibility, sequence_mask  # noqa: F401  (train_standalone.py:227-234, 328-333)


def normalize(data, mu, std):
    """train_standalone.py:204-224: (data - mu) / std, mu / std scalars or per-channel lists / tensors / arrays"""
    import numpy as np

    def per_channel(v):
        if isinstance(v, (float, int)):
            return v
        if isinstance(v, list):
            v = torch.tensor(v, dtype=data.dtype, device=data.device)
        elif isinstance(v, np.ndarray):
            v = torch.from_numpy(v).to(data.device)
        elif isinstance(v, torch.Tensor):
            v = v.to(data.device)
        return v.unsqueeze(-1)

    return (data - per_channel(mu)) / per_channel(std)


def duration_loss(logw, logw_, lengths):
    """train_standalone.py:336-339"""
    return torch.sum((logw - logw_) ** 2) / torch.sum(lengths)


def maximum_path(neg_cent, mask):
    """train_standalone.py:280-325 (Monotonic Alignment Search) on the GPU: mt_maximum_path"""
    return rt.maximum_path(neg_cent, mask)


def _get(p, k, default=None):
    return p.get(k, default) if isinstance(p, dict) else getattr(p, k, default)


class _FusedAdam:
    """configure_optimizers' Adam(lr) with Lightning's gradient_clip_val = 5.0 folded in: one clip-factor kernel
    and one Adam kernel over the flat parameter buffer. ``state_dict`` / ``load_state_dict`` use torch.optim.Adam's
    format over ``module.parameters()`` (per-parameter exp_avg / exp_avg_sq / step), so a resumed run continues with
    the moments and the step count it saved."""

    def __init__(self, module: "MatchaLightningModule"):
        self.module = module
        self.param_groups = [{"lr": module.learning_rate, "betas": (0.9, 0.999), "eps": 1e-8, "weight_decay": 0,
                              "amsgrad": False, "maximize": False}]
        self._pending = None  # a loaded state not yet applied (the trainer is built on first use)

    def step(self, closure=None):
        if closure is not None:
            raise NotImplementedError("closures are not supported")
        tr = self.module.trainer()
        tr.lr = float(self.param_groups[0]["lr"])
        tr.optimizer_step()
        self.module._sync_model()

    def zero_grad(self, set_to_none: bool = True):
        pass  # every backward overwrites the whole flat gradient buffer

    def _index(self):
        """module.parameters() order -> trainer parameter name (the reference's Adam state is keyed by it)"""
        names = [n for n, _ in self.module.named_parameters()]
        return [n[len("model."):] if n.startswith("model.") else n for n in names]

    def state_dict(self):
        tr = self.module.trainer()
        st = tr.optimizer_state()
        m_view = {n: st["exp_avg"][o:o + k] for n, o, k in tr.grads.spans}
        v_view = {n: st["exp_avg_sq"][o:o + k] for n, o, k in tr.grads.spans}
        state = {}
        for i, n in enumerate(self._index()):
            if n in m_view and st["step"] > 0:
                shape = tr.params.view[n].shape
                state[i] = {"step": torch.tensor(float(st["step"])), "exp_avg": m_view[n].view(shape).clone(),
                            "exp_avg_sq": v_view[n].view(shape).clone()}
        # the engine's dropout-stream position rides in the param group (torch's Adam keeps only hyper-parameters
        # there; an extra key is carried through load_state_dict unchanged)
        groups = [dict(self.param_groups[0], params=list(range(len(self._index()))), dropout_calls=int(st["calls"]))]
        if st.get("scaler") is not None:  # "16-mixed": GradScaler.state_dict() (Lightning checkpoints it too)
            groups[0]["loss_scaler"] = dict(st["scaler"])
        return {"state": state, "param_groups": groups}

    def load_state_dict(self, sd):
        """applied to the training engine before its next use (it is built on the device on first use)"""
        self.param_groups[0].update({k: v for k, v in sd["param_groups"][0].items() if k != "params"})
        self._pending = sd
        self.module._pending_opt = self

    @torch.no_grad()
    def _apply_pending(self, tr):
        if self._pending is None:
            return
        sd, self._pending = self._pending, None
        m, v = torch.zeros_like(tr.m), torch.zeros_like(tr.v)
        spans = {n: (o, k) for n, o, k in tr.grads.spans}
        step = 0
        for i, n in enumerate(self._index()):
            st = sd["state"].get(i) if isinstance(sd["state"], dict) else None
            if st is None or n not in spans:
                continue
            o, k = spans[n]
            m[o:o + k].copy_(st["exp_avg"].reshape(-1))
            v[o:o + k].copy_(st["exp_avg_sq"].reshape(-1))
            step = int(float(st["step"]))
        tr.load_optimizer_state({"exp_avg": m, "exp_avg_sq": v, "step": step,
                                 "lr": self.param_groups[0]["lr"],
                                 "calls": sd["param_groups"][0].get("dropout_calls"),
                                 "scaler": sd["param_groups"][0].get("loss_scaler")})


class MatchaLightningModule(torch.nn.Module):
    """train_standalone.py:580-707 (single speaker). ``forward`` returns (dur_loss, prior_loss, cfm_loss, attn) like
    the reference; in training mode it also runs the backward, leaving the gradients for ``optimizer.step()``."""

    def __init__(self, n_vocab, n_spks, spk_emb_dim, encoder_params, decoder_params, cfm_params,
                 duration_predictor_params, data_statistics, learning_rate=1e-4, prior_loss=True,
                 process_group=None, precision="32"):
        super().__init__()
        if n_spks > 1:
            raise NotImplementedError("multi-speaker training (spk_emb conditioning) is not built")
        self.learning_rate, self.n_vocab, self.n_spks = learning_rate, n_vocab, n_spks
        self.n_feats = _get(encoder_params, "n_feats")
        self.prior_loss = prior_loss
        # dropout rates of the configs (train_standalone.py:772-800); the prenet's 0.5 is fixed (model.py:481)
        self.p_dropout = {"encoder": float(_get(encoder_params, "p_dropout", 0.1)),
                          "duration_predictor": float(_get(duration_predictor_params, "p_dropout", 0.1)),
                          "decoder": float(_get(decoder_params, "dropout", 0.05))}
        self.hp = {"n_layers": _get(encoder_params, "n_layers"), "n_heads": _get(encoder_params, "n_heads"),
                   "n_spks": n_spks}
        self.heads = _get(decoder_params, "num_heads", 2)
        self.sigma_min = _get(cfm_params, "sigma_min", 1e-4)
        self.model = _model.MatchaTTS(n_vocab, n_spks, spk_emb_dim, encoder_params, decoder_params, cfm_params,
                                      duration_predictor_params)
        self.register_buffer("mel_mean", torch.tensor(data_statistics["mel_mean"]))
        self.register_buffer("mel_std", torch.tensor(data_statistics["mel_std"]))
        self.model.mel_mean = self.mel_mean
        self.model.mel_std = self.mel_std
        self.process_group = process_group
        # the reference sets this on pl.Trainer (precision="16-mixed", train_standalone.py:868); the engine lives
        # here, so the module takes it: "32", "16-mixed" (fp16 operands + dynamic loss scale) or "bf16-mixed"
        self.precision = str(precision)
        self._tr: Optional[MatchaTrainer] = None
        self._fp = None  # (address, version) of the model's tensors when the trainer last matched them
        self._pending_opt: Optional[_FusedAdam] = None  # an optimizer state loaded before the engine existed
        self.logged = {}

    def _world(self) -> int:
        return dist.get_world_size(self.process_group) if dist.is_available() and dist.is_initialized() else 1

    def _model_fp(self):
        """(address, version) of the tensors the engine holds (the buffers mel_mean / mel_std are not among them:
        _broadcast_buffers rewrites those every DDP step and must not trigger a parameter reload)"""
        return [(t.data_ptr(), t._version) for k, t in self.model.state_dict(keep_vars=True).items()
                if k.startswith(("encoder.", "decoder.estimator."))]

    def trainer(self) -> MatchaTrainer:
        """the GPU training engine, built from the model's current weights on first use; a later change of the
        model's weights from outside (load_state_dict on this module or on .model, an in-place edit) is copied
        into it before its next use (the Adam moments are kept)"""
        dev = self.mel_mean.device
        if self._tr is None or self._tr.params.flat.device != dev:
            rt.require_gpu(self.mel_mean, what="MatchaLightningModule")
            self._tr = MatchaTrainer(self.model.state_dict(), self.hp, dev, lr=self.learning_rate,
                                     sigma_min=self.sigma_min, prior_loss=self.prior_loss, heads=self.heads,
                                     process_group=self.process_group, p_dropout=self.p_dropout,
                                     precision=self.precision)
            if self._tr.world > 1:
                self._sync_model()  # the ranks' modules hold rank 0's weights, as under DDP
            self._fp = self._model_fp()
        elif self._model_fp() != self._fp:
            self._tr.load_parameters(self.model.state_dict())
            self._fp = self._model_fp()
        if self._pending_opt is not None:
            opt, self._pending_opt = self._pending_opt, None
            opt._apply_pending(self._tr)
        return self._tr

    @torch.no_grad()
    def _sync_model(self):
        sd = self.model.state_dict(keep_vars=True)
        for k, v in self._tr.parameters().items():
            sd[k].data.copy_(v)
        self._fp = self._model_fp()

    @torch.no_grad()
    def _broadcast_buffers(self):
        """DDP broadcast_buffers (default True): rank 0's buffers before every forward — every buffer of the module
        tree (mel_mean / mel_std here and in .model: `.to()` gives each module its own copy), as one message"""
        if self._world() > 1:
            src = dist.get_global_rank(self.process_group, 0) if self.process_group else 0
            bufs = list(self.buffers())
            flat = torch.cat([b.detach().reshape(-1).to(torch.float32) for b in bufs])
            dist.broadcast(flat, src=src, group=self.process_group)
            o = 0
            for b in bufs:
                b.copy_(flat[o:o + b.numel()].view(b.shape))
                o += b.numel()

    def _log(self, prefix, loss, dur, prior, cfm):
        """self.log(..., sync_dist=True) (train_standalone.py:680-683, 698-701): the mean over the DDP ranks"""
        vals = torch.stack([loss, dur, prior, cfm]).detach().float()
        if self._world() > 1:
            dist.all_reduce(vals, op=dist.ReduceOp.SUM, group=self.process_group)
            vals = vals / self._world()
        self.logged.update({f"{prefix}/loss": vals[0], f"{prefix}/dur_loss": vals[1],
                            f"{prefix}/prior_loss": vals[2], f"{prefix}/cfm_loss": vals[3]})

    def forward(self, x, x_lengths, y, y_lengths, spks=None):
        if spks is not None and self.n_spks > 1:
            raise NotImplementedError("multi-speaker training (spk_emb conditioning) is not built")
        self._broadcast_buffers()
        tr = self.trainer().set_dropout(self.training)
        out = tr.forward_backward(x, x_lengths, y, y_lengths, backward=self.training)
        # attn: maximum_path's [B, T_x, T_y] as the reference returns it (train_standalone.py:646, 667)
        return out["dur_loss"][0], out["prior_loss"][0], out["cfm_loss"][0], out["attn"]

    def training_step(self, batch, batch_idx):
        """train_standalone.py:669-685 -> loss; logs train/{loss,dur_loss,prior_loss,cfm_loss} into self.logged"""
        self.train()
        dur, prior, cfm, _ = self(batch["x"], batch["x_lengths"], batch["y"], batch["y_lengths"], batch.get("spks"))
        loss = dur + prior + cfm
        self._log("train", loss, dur, prior, cfm)
        return loss

    @torch.no_grad()
    def validation_step(self, batch, batch_idx):
        """train_standalone.py:687-703 (eval-mode dropout, no backward)"""
        was = self.training
        self.eval()
        try:
            dur, prior, cfm, _ = self(batch["x"], batch["x_lengths"], batch["y"], batch["y_lengths"],
                                      batch.get("spks"))
        finally:
            self.train(was)
        loss = dur + prior + cfm
        self._log("val", loss, dur, prior, cfm)
        return loss

    def configure_optimizers(self):
        """train_standalone.py:705-707 (Adam, lr) with the Trainer's gradient_clip_val 5.0"""
        return _FusedAdam(self)
