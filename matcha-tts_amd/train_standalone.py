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

import model as _model
from hifigan.meldataset import mel_spectrogram, normalize  # noqa: F401  (train_standalone.py:164-224)
from matcha_hip import runtime as rt
from matcha_hip.train import MatchaTrainer
from model import fix_len_compatibility, sequence_mask  # noqa: F401  (train_standalone.py:227-234, 328-333)


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
    and one Adam kernel over the flat parameter buffer."""

    def __init__(self, module: "MatchaLightningModule"):
        self.module = module
        self.param_groups = [{"lr": module.learning_rate, "betas": (0.9, 0.999), "eps": 1e-8, "weight_decay": 0}]

    def step(self, closure=None):
        if closure is not None:
            raise NotImplementedError("closures are not supported")
        tr = self.module.trainer()
        tr.lr = float(self.param_groups[0]["lr"])
        tr.optimizer_step()
        self.module._sync_model()

    def zero_grad(self, set_to_none: bool = True):
        pass  # every backward overwrites the whole flat gradient buffer


class MatchaLightningModule(torch.nn.Module):
    """train_standalone.py:580-707 (single speaker). ``forward`` returns (dur_loss, prior_loss, cfm_loss, attn) like
    the reference; in training mode it also runs the backward, leaving the gradients for ``optimizer.step()``."""

    def __init__(self, n_vocab, n_spks, spk_emb_dim, encoder_params, decoder_params, cfm_params,
                 duration_predictor_params, data_statistics, learning_rate=1e-4, prior_loss=True,
                 process_group=None):
        super().__init__()
        if n_spks > 1:
            raise NotImplementedError("multi-speaker training (spk_emb conditioning) is not built")
        self.learning_rate, self.n_vocab, self.n_spks = learning_rate, n_vocab, n_spks
        self.n_feats = _get(encoder_params, "n_feats")
        self.prior_loss = prior_loss
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
        self._tr: Optional[MatchaTrainer] = None
        self.logged = {}

    def trainer(self) -> MatchaTrainer:
        """the GPU training engine, built from the model's current weights on first use"""
        dev = self.mel_mean.device
        if self._tr is None or self._tr.params.flat.device != dev:
            rt.require_gpu(self.mel_mean, what="MatchaLightningModule")
            self._tr = MatchaTrainer(self.model.state_dict(), self.hp, dev, lr=self.learning_rate,
                                     sigma_min=self.sigma_min, prior_loss=self.prior_loss, heads=self.heads,
                                     process_group=self.process_group)
        return self._tr

    @torch.no_grad()
    def _sync_model(self):
        sd = self.model.state_dict(keep_vars=True)
        for k, v in self._tr.parameters().items():
            sd[k].data.copy_(v)

    def forward(self, x, x_lengths, y, y_lengths, spks=None):
        if spks is not None and self.n_spks > 1:
            raise NotImplementedError("multi-speaker training (spk_emb conditioning) is not built")
        tr = self.trainer().set_dropout(self.training)
        out = tr.forward_backward(x, x_lengths, y, y_lengths, backward=self.training)
        return out["dur_loss"][0], out["prior_loss"][0], out["cfm_loss"][0], out["attn"].unsqueeze(1)

    def training_step(self, batch, batch_idx):
        """train_standalone.py:669-685 -> loss; logs train/{loss,dur_loss,prior_loss,cfm_loss} into self.logged"""
        self.train()
        dur, prior, cfm, _ = self(batch["x"], batch["x_lengths"], batch["y"], batch["y_lengths"], batch.get("spks"))
        loss = dur + prior + cfm
        self.logged.update({"train/loss": loss, "train/dur_loss": dur, "train/prior_loss": prior,
                            "train/cfm_loss": cfm})
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
        self.logged.update({"val/loss": loss, "val/dur_loss": dur, "val/prior_loss": prior, "val/cfm_loss": cfm})
        return loss

    def configure_optimizers(self):
        """train_standalone.py:705-707 (Adam, lr) with the Trainer's gradient_clip_val 5.0"""
        return _FusedAdam(self)
