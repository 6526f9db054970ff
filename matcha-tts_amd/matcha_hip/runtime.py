"""Host runtime over the C ABI: handles, packed-weight caches and workspaces.

PyTorch owns every device buffer (inputs, outputs, packed weights, workspaces); the
library only enqueues kernels on the current stream. All entry points require CUDA
(ROCm) tensors and raise ``HipPathError`` otherwise — there is no CPU fallback.
"""
from __future__ import annotations

import math
import time
from ctypes import byref, c_char_p, c_int, c_int64, c_void_p, create_string_buffer
from typing import Dict, List, Optional, Tuple

import torch

from ._lib import (DTYPE_BF16, DTYPE_F32, SOLVER_EULER, SOLVER_MIDPOINT, HipPathError, check, lib,
                   ptr, stream_handle)

_DTYPES = {"fp32": DTYPE_F32, "float32": DTYPE_F32, "f32": DTYPE_F32,
           "bf16": DTYPE_BF16, "bfloat16": DTYPE_BF16,
           # text encoder only: fp32 storage and arithmetic, the FFN convs' products as six bf16 MFMA products of
           # 3-way bf16 splits (mt_encoder_set_split)
           "fp32x3": DTYPE_F32}


def dtype_code(precision: str) -> int:
    try:
        return _DTYPES[precision]
    except KeyError:
        raise ValueError(f"precision must be one of {sorted(set(_DTYPES))}, got {precision!r}")


def require_gpu(*tensors, what: str = "matcha_hip") -> None:
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise HipPathError(
                f"{what}: the synthesis path runs on the MI355X (ROCm) device only; got a tensor on "
                f"{t.device}. Move the model and inputs to 'cuda'.")


def f32c(t: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    if t is None:
        return None
    return t.detach().to(torch.float32).contiguous()


class _Workspace:
    """Grow-only device scratch per (device, stream)."""

    _bufs: Dict[Tuple[int, int], torch.Tensor] = {}

    @classmethod
    def get(cls, nbytes: int, device: torch.device) -> torch.Tensor:
        key = (device.index if device.index is not None else torch.cuda.current_device(),
               stream_handle(device))
        buf = cls._bufs.get(key)
        if buf is None or buf.numel() < nbytes:
            cls._bufs.pop(key, None)
            buf = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=device)
            cls._bufs[key] = buf
        return buf


def _param_list(h, num_fn, name_fn, shape_fn) -> List[Tuple[str, Tuple[int, ...]]]:
    L = lib()
    n = getattr(L, num_fn)(h)
    out = []
    buf = create_string_buffer(256)
    shp = (c_int64 * 8)()
    for i in range(n):
        check(getattr(L, name_fn)(h, i, buf, 256), name_fn)
        nd = getattr(L, shape_fn)(h, i, shp, 8)
        if nd < 0:
            check(nd, shape_fn)
        out.append((buf.value.decode(), tuple(int(shp[k]) for k in range(nd))))
    return out


# Every parameter / buffer / submodule (re)registration anywhere bumps this counter (torch's global
# module registration hooks), so PackCache reuses a packed buffer only while no registration happened
# and the module's state tensors are the same tensors at the same addresses and version counters.
_REG = [0]


def _bump_registration(*_args):
    _REG[0] += 1


for _hook in (torch.nn.modules.module.register_module_parameter_registration_hook,
              torch.nn.modules.module.register_module_buffer_registration_hook,
              torch.nn.modules.module.register_module_module_registration_hook):
    _hook(_bump_registration)


class PackCache:
    """Per-module cache of packed weight buffers, keyed by (precision, device).

    A hit costs one pass over the module's state tensors (address + version counter); a miss (first call,
    in-place weight update, `param.data = ...`, a registration such as remove_weight_norm, .to()) makes
    the caller rebuild state_dict() and repack. `trust_next` lets one internal call sequence (synthesize)
    validate early, while the GPU is still busy, and skip the check at the point of use."""

    def __init__(self):
        self.entries = {}
        self.trusted = set()

    def get(self, key):
        e = self.entries.get(key)
        if e is None:
            return None
        if key in self.trusted:
            self.trusted.discard(key)
            return e[3]
        reg, tensors, state, packed = e
        if reg != _REG[0] or [(t.data_ptr(), t._version) for t in tensors] != state:
            return None
        return packed

    def put(self, key, tensors, packed):
        self.entries[key] = (_REG[0], tensors, [(t.data_ptr(), t._version) for t in tensors], packed)
        return packed

    def trust_next(self, key):
        if key in self.entries:
            self.trusted.add(key)

    def untrust(self):
        self.trusted.clear()


def fingerprint(tensors: List[torch.Tensor]) -> Tuple:
    return tuple((t.data_ptr(), t._version, tuple(t.shape), str(t.device)) for t in tensors)


def sinus_freq(c_cond: int) -> torch.Tensor:
    """model.py:757-759 frequency table, formed exactly as the reference does (fp32, CPU)."""
    half = c_cond // 2
    e = math.log(10000) / (half - 1)
    return torch.exp(torch.arange(half).float() * -e)


def rope_theta(head_dim: int) -> torch.Tensor:
    """model.py:258-265 theta table, formed exactly as the reference does (fp32, CPU)."""
    d = int(head_dim * 0.5)
    return 1.0 / (10_000 ** (torch.arange(0, d, 2).float() / d))


class EncoderEngine:
    """mt_encoder handle: text encoder + duration predictor (model.py:452-535) for one config/dtype."""

    def __init__(self, n_vocab: int, n_channels: int, filter_channels: int, n_heads: int, n_layers: int,
                 kernel_size: int, n_spks: int, spk_emb_dim: int, dp_filter: int, dp_kernel: int, prenet: bool,
                 precision: str):
        self.dtype = dtype_code(precision)
        self.width = n_channels + (spk_emb_dim if n_spks > 1 else 0)
        self.head_dim = self.width // n_heads
        h = c_void_p()
        check(lib().mt_encoder_create(n_vocab, n_channels, filter_channels, n_heads, n_layers, kernel_size, n_spks,
                                      spk_emb_dim, dp_filter, dp_kernel, int(bool(prenet)), self.dtype, byref(h)),
              "encoder_create")
        self.h = h
        self.specs = _param_list(h, "mt_encoder_num_params", "mt_encoder_param_name", "mt_encoder_param_shape")
        self.packed_bytes = lib().mt_encoder_packed_bytes(h)
        self._packed = None
        self._fp = None
        if precision == "fp32x3":
            self.set_split(True)

    def __del__(self):
        try:
            if getattr(self, "h", None):
                lib().mt_encoder_destroy(self.h)
        except Exception:
            pass

    def set_mfma_attention(self, enable) -> None:
        """bf16, 96-dim heads: attention core on MFMA (1, default) or on the fp32-VALU kernel (0)."""
        check(lib().mt_encoder_set_mfma_attention(self.h, int(bool(enable))), "encoder_set_mfma_attention")

    def set_vconv(self, enable) -> None:
        """fp32: convs on mt_vconv's fp32 mode (1, default) or on the generic conv kernel (0)."""
        check(lib().mt_encoder_set_vconv(self.h, int(bool(enable))), "encoder_set_vconv")

    def set_split(self, enable) -> None:
        """fp32: the FFN convs on mt_vconv's split-bf16 mode (1; precision "fp32x3") or exact fp32 MFMA (0)."""
        check(lib().mt_encoder_set_split(self.h, int(bool(enable))), "encoder_set_split")

    def pack(self, params: Dict[str, torch.Tensor], device: torch.device) -> torch.Tensor:
        """params: TextEncoder-relative reference keys -> tensors."""
        tensors = []
        for name, shape in self.specs:
            t = rope_theta(self.head_dim) if name == "_rope_theta" else params.get(name)
            if t is None:
                raise KeyError(f"text encoder parameter {name!r} missing")
            if tuple(t.shape) != shape:
                raise ValueError(f"{name}: shape {tuple(t.shape)} != expected {shape}")
            tensors.append(t)
        fp = fingerprint([t for (n, _), t in zip(self.specs, tensors) if n != "_rope_theta"]) + (str(device),)
        if self._packed is not None and fp == self._fp:
            return self._packed
        dev = [t.detach().to(device=device, dtype=torch.float32).contiguous() for t in tensors]
        packed = torch.empty(self.packed_bytes, dtype=torch.uint8, device=device)
        arr = (c_void_p * len(dev))(*[t.data_ptr() for t in dev])
        check(lib().mt_encoder_pack(self.h, arr, packed.data_ptr(), stream_handle(device)), "encoder_pack")
        torch.cuda.current_stream(device).synchronize()  # staging copies die with `dev`
        self._packed, self._fp = packed, fp
        return packed

    def forward(self, packed, x: torch.Tensor, x_lengths: torch.Tensor, spks: Optional[torch.Tensor] = None):
        """x int64 [B,Tx], x_lengths int64 [B] -> mu [B,80,Tx], logw [B,1,Tx], x_mask [B,1,Tx] (fp32), oov int32 [1]
        (1 when an id of x lies outside [0, n_vocab): see ``check_ids``)."""
        x = x.to(torch.int64).contiguous()
        xl = x_lengths.to(torch.int64).contiguous()
        B, Tx = x.shape
        dev = x.device
        mu = torch.empty(B, 80, Tx, dtype=torch.float32, device=dev)
        logw = torch.empty(B, 1, Tx, dtype=torch.float32, device=dev)
        x_mask = torch.empty(B, 1, Tx, dtype=torch.float32, device=dev)
        L = lib()
        oov = torch.empty(1, dtype=torch.int32, device=dev)
        ws = _Workspace.get(L.mt_encoder_workspace_bytes(self.h, B, Tx), dev)
        check(L.mt_encoder_forward(self.h, packed.data_ptr(), ptr(x), ptr(xl), ptr(spks), B, Tx, ptr(mu), ptr(logw),
                                   ptr(x_mask), ptr(oov), ws.data_ptr(), ws.numel(), stream_handle(dev)),
              "encoder_forward")
        return mu, logw, x_mask, oov


def check_ids(oov: torch.Tensor) -> None:
    """nn.Embedding's error for an out-of-vocabulary token id (model.py:471, 522: ``self.emb(x)`` raises
    IndexError on the CPU; on a GPU torch reports it at the next sync). Reads the encoder's device flag, i.e. one
    host sync: ``MatchaTTS.synthesize`` calls it right after the reference's own sync on max(y_lengths)."""
    if int(oov.item()) != 0:
        raise IndexError("index out of range in self (a token id of x lies outside [0, n_vocab))")


class DecoderEngine:
    """mt_decoder handle: U-Net estimator + CFM solver for one (c_cond, dtype)."""

    def __init__(self, c_cond: int, n_mid: int, n_blocks: int, heads: int, precision: str):
        self.c_cond, self.dtype = c_cond, dtype_code(precision)
        h = c_void_p()
        check(lib().mt_decoder_create(c_cond, n_mid, n_blocks, heads, self.dtype, byref(h)),
              "decoder_create")
        self.h = h
        self.specs = _param_list(h, "mt_decoder_num_params", "mt_decoder_param_name",
                                 "mt_decoder_param_shape")
        self.packed_bytes = lib().mt_decoder_packed_bytes(h)
        self._packed = None
        self._fp = None

    def __del__(self):
        try:
            if getattr(self, "h", None):
                lib().mt_decoder_destroy(self.h)
        except Exception:
            pass

    def pack(self, params: Dict[str, torch.Tensor], device: torch.device) -> torch.Tensor:
        """params: estimator-relative reference keys -> tensors (any device/dtype)."""
        tensors = []
        for name, shape in self.specs:
            if name == "_sinus_freq":
                t = sinus_freq(self.c_cond)
            else:
                if name not in params:
                    raise KeyError(f"estimator parameter {name!r} missing")
                t = params[name]
            if tuple(t.shape) != shape:
                raise ValueError(f"{name}: shape {tuple(t.shape)} != expected {shape}")
            tensors.append(t)
        fp = fingerprint([t for (n, _), t in zip(self.specs, tensors) if n != "_sinus_freq"]) + (str(device),)
        if self._packed is not None and fp == self._fp:
            return self._packed
        dev = [t.detach().to(device=device, dtype=torch.float32).contiguous() for t in tensors]
        packed = torch.empty(self.packed_bytes, dtype=torch.uint8, device=device)
        arr = (c_void_p * len(dev))(*[t.data_ptr() for t in dev])
        check(lib().mt_decoder_pack(self.h, arr, packed.data_ptr(), stream_handle(device)), "decoder_pack")
        torch.cuda.current_stream(device).synchronize()  # staging copies die with `dev`
        self._packed, self._fp = packed, fp
        return packed

    def set_vconv(self, mode) -> None:
        """bf16: 1 (default) ResnetBlock / down / up / final convs on mt_vconv with block 2's GroupNorm + Mish
        in the res conv's epilogue; 2 the same with that GroupNorm as a separate pass; 0 generic conv kernel.
        True / False map to 1 / 0."""
        check(lib().mt_decoder_set_vconv(self.h, int(mode)), "decoder_set_vconv")

    def set_uniform_attention(self, enable) -> None:
        """1 (default): query-independent attention where the caller's max_valid proves every utterance padded."""
        check(lib().mt_decoder_set_uniform_attention(self.h, int(bool(enable))), "decoder_set_uniform_attention")

    def set_graphs(self, enable) -> None:
        """1 (default): solve() replays its evaluation chain as a cached hipGraph; 0: direct launches."""
        check(lib().mt_decoder_set_graphs(self.h, int(bool(enable))), "decoder_set_graphs")

    def solve(self, packed, z_noise, temperature, mu_y, mask, spks, n_timesteps, solver="euler",
              out=None, max_valid: int = 0):
        """max_valid: the most valid frames of any utterance (synthesize's y_max), 0 when unknown."""
        B, C, T = mu_y.shape
        s = SOLVER_EULER if solver == "euler" else SOLVER_MIDPOINT if solver == "midpoint" else None
        if s is None:
            raise NotImplementedError(f"Solver {solver} not implemented")
        out = torch.empty_like(mu_y) if out is None else out
        L = lib()
        nbytes = L.mt_cfm_workspace_bytes(self.h, B, T, n_timesteps, s)
        ws = _Workspace.get(nbytes, mu_y.device)
        check(L.mt_cfm_solve_bounded(self.h, packed.data_ptr(), ptr(z_noise), float(temperature), ptr(mu_y),
                                     ptr(mask), ptr(spks), B, T, int(max_valid), int(n_timesteps), s, ptr(out),
                                     ws.data_ptr(), ws.numel(), stream_handle(mu_y.device)), "cfm_solve")
        return out

    TAPS = ("down0_res", "down0_tb", "mid1_tb", "up0_out", "up1_tb")

    def step_taps(self, packed, x, mu_y, mask, spks, t: float):
        """One evaluation plus the block outputs of DecoderEngine.TAPS as fp32 [B,256,T_l] (mt_decoder_set_taps)."""
        B, _, T = mu_y.shape
        taps = [torch.empty((B, 256, T // 2 if n == "mid1_tb" else T), dtype=torch.float32, device=mu_y.device)
                for n in self.TAPS]
        arr = (c_void_p * len(taps))(*[t_.data_ptr() for t_ in taps])
        check(lib().mt_decoder_set_taps(self.h, arr, len(taps)), "decoder_set_taps")
        try:
            out = self.step(packed, x, mu_y, mask, spks, t)
            torch.cuda.current_stream(mu_y.device).synchronize()
        finally:
            check(lib().mt_decoder_set_taps(self.h, None, 0), "decoder_set_taps")
        return out, dict(zip(self.TAPS, taps))

    def step(self, packed, x, mu_y, mask, spks, t: float, out=None):
        B, C, T = mu_y.shape
        out = torch.empty_like(mu_y) if out is None else out
        L = lib()
        nbytes = L.mt_decoder_step_workspace_bytes(self.h, B, T)
        ws = _Workspace.get(nbytes, mu_y.device)
        check(L.mt_decoder_step(self.h, packed.data_ptr(), ptr(x), ptr(mu_y), ptr(mask), ptr(spks), float(t),
                                B, T, ptr(out), ws.data_ptr(), ws.numel(), stream_handle(mu_y.device)),
              "decoder_step")
        return out


    def step_times(self, packed, x, mu_y, mask, spks, t: torch.Tensor, out=None):
        """One evaluation with a time per utterance: t [B] (device)."""
        B, C, T = mu_y.shape
        out = torch.empty_like(mu_y) if out is None else out
        tt = f32c(t.reshape(-1).to(mu_y.device))
        if tt.numel() != B:
            raise ValueError(f"t has {tt.numel()} values for a batch of {B}")
        L = lib()
        ws = _Workspace.get(L.mt_decoder_step_times_workspace_bytes(self.h, B, T), mu_y.device)
        check(L.mt_decoder_step_times(self.h, packed.data_ptr(), ptr(x), ptr(mu_y), ptr(mask), ptr(spks), ptr(tt),
                                      B, T, ptr(out), ws.data_ptr(), ws.numel(), stream_handle(mu_y.device)),
              "decoder_step_times")
        return out


class VocoderEngine:
    """mt_vocoder handle: HiFi-GAN Generator for one config and dtype."""

    def __init__(self, h: dict, precision: str):
        self.dtype = dtype_code(precision)
        ur, uk = list(h["upsample_rates"]), list(h["upsample_kernel_sizes"])
        rk = list(h["resblock_kernel_sizes"])
        rd = [list(d) for d in h["resblock_dilation_sizes"]]
        nd = len(rd[0])
        if any(len(d) != nd for d in rd):
            raise ValueError("resblock dilation lists must have equal length")
        flat = [x for d in rd for x in d]
        ci = lambda v: (c_int * len(v))(*v)  # noqa: E731
        hdl = c_void_p()
        check(lib().mt_vocoder_create(1 if str(h["resblock"]) == "1" else 2, len(ur), ci(ur), ci(uk),
                                      int(h["upsample_initial_channel"]), len(rk), ci(rk), nd, ci(flat),
                                      self.dtype, byref(hdl)), "vocoder_create")
        self.h = hdl
        self.hop = int(math.prod(ur))
        self.specs = _param_list(hdl, "mt_vocoder_num_params", "mt_vocoder_param_name",
                                 "mt_vocoder_param_shape")
        self.packed_bytes = lib().mt_vocoder_packed_bytes(hdl)
        self._packed = None
        self._fp = None

    def set_fusion(self, enable: bool) -> None:
        check(lib().mt_vocoder_set_fusion(self.h, int(bool(enable))), "vocoder_set_fusion")

    def set_pair(self, mode) -> None:
        """bf16 ResBlock pairs as one launch each: 1 (default) the 64- / 32-channel stages and the 128-channel
        stage's k = 3 resblock; 4 every 128-channel pair too; 2 none of the 128-channel stage; 0 all per layer."""
        check(lib().mt_vocoder_set_pair(self.h, int(mode)), "vocoder_set_pair")

    def set_vconv(self, mode) -> None:
        """0 generic per-layer kernel, 1 vconv for the 128/256-channel stages, 2 (default) also for 64."""
        check(lib().mt_vocoder_set_vconv(self.h, int(mode)), "vocoder_set_vconv")

    def __del__(self):
        try:
            if getattr(self, "h", None):
                lib().mt_vocoder_destroy(self.h)
        except Exception:
            pass

    def pack(self, params_fn, src: List[torch.Tensor], device: torch.device) -> torch.Tensor:
        """params_fn() -> folded reference-keyed weights; repacked only when ``src`` changes."""
        fp = fingerprint(src) + (str(device),)
        if self._packed is not None and fp == self._fp:
            return self._packed
        params = params_fn()
        tensors = []
        for name, shape in self.specs:
            if name not in params:
                raise KeyError(f"vocoder parameter {name!r} missing")
            t = params[name]
            if tuple(t.shape) != shape:
                raise ValueError(f"{name}: shape {tuple(t.shape)} != expected {shape}")
            tensors.append(t)
        dev = [t.detach().to(device=device, dtype=torch.float32).contiguous() for t in tensors]
        packed = torch.empty(self.packed_bytes, dtype=torch.uint8, device=device)
        arr = (c_void_p * len(dev))(*[t.data_ptr() for t in dev])
        check(lib().mt_vocoder_pack(self.h, arr, packed.data_ptr(), stream_handle(device)), "vocoder_pack")
        torch.cuda.current_stream(device).synchronize()
        self._packed, self._fp = packed, fp
        return packed

    def ragged_supported(self) -> bool:
        return bool(lib().mt_vocoder_ragged_supported(self.h))

    def forward(self, packed, mel, out=None, lengths=None):
        """lengths (int [B], mel frames, or None): a ragged batch, utterance b vocoded at its own lengths[b]
        frames (mt_vocoder_forward_ragged); its samples past hop * lengths[b] are zero"""
        B, C, T = mel.shape
        out = torch.empty((B, 1, T * self.hop), dtype=torch.float32, device=mel.device) if out is None else out
        L = lib()
        ws = _Workspace.get(L.mt_vocoder_workspace_bytes(self.h, B, T), mel.device)
        if lengths is None:
            check(L.mt_vocoder_forward(self.h, packed.data_ptr(), ptr(mel), B, T, ptr(out), ws.data_ptr(),
                                       ws.numel(), stream_handle(mel.device)), "vocoder_forward")
            return out
        lens = lengths.to(device=mel.device, dtype=torch.int32).contiguous()
        if lens.shape != (B,):
            raise ValueError(f"lengths {tuple(lens.shape)}: expected ({B},)")
        check(L.mt_vocoder_forward_ragged(self.h, packed.data_ptr(), ptr(mel), B, T, ptr(lens), ptr(out),
                                          ws.data_ptr(), ws.numel(), stream_handle(mel.device)), "vocoder_forward")
        return out


# ---- index path / small ops ---------------------------------------------------------------

# utterances one ragged vocoder launch chain takes (mt_ragged.h RAG_MAXB: the per-utterance tile table lives in LDS);
# Generator.forward splits larger batches (tests/test_abi_host.py checks the two stay equal)
RAGGED_MAX_BATCH = 512

_HOST_BUFS: Dict[tuple, torch.Tensor] = {}


def fetch_ints(t: torch.Tensor) -> List[int]:
    """A few device int64 values -> Python ints (synthesize's one host sync, model.py:1278-1281): an async copy into
    a pinned buffer, then the host polls the copy's event. A blocking wait lets the host thread sleep, and its
    wake-up left the GPU idle ≈ 0.16 ms between the durations and the alignment kernels in the B = 32 bench trace
    (profiles/r06b_kernel_stats.csv's step)."""
    import threading
    n = t.numel()
    key = (str(t.device), n, threading.get_ident())
    buf = _HOST_BUFS.get(key)
    if buf is None:
        buf = _HOST_BUFS[key] = torch.empty(n, dtype=torch.int64, pin_memory=True)
    buf.copy_(t.reshape(-1).to(torch.int64), non_blocking=True)
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(t.device))
    polls = 0
    while not ev.query():
        polls += 1
        if polls > 256:  # past the first ~0.5 ms: yield the core between polls (a long encoder at large B)
            time.sleep(0)
    return buf.tolist()


def durations(logw: torch.Tensor, x_mask: torch.Tensor, length_scale: float):
    """model.py:1273-1275 -> (w_ceil [B,1,Tx], cum [B,Tx], y_lengths int64 [B])."""
    require_gpu(logw, x_mask, what="durations")
    logw, x_mask = f32c(logw), f32c(x_mask)
    B, _, Tx = logw.shape
    w_ceil = torch.empty((B, 1, Tx), dtype=torch.float32, device=logw.device)
    cum = torch.empty((B, Tx), dtype=torch.float32, device=logw.device)
    yl = torch.empty((B,), dtype=torch.int64, device=logw.device)
    check(lib().mt_durations(ptr(logw), ptr(x_mask), float(length_scale), B, Tx, ptr(w_ceil), ptr(cum),
                             ptr(yl), stream_handle(logw.device)), "durations")
    return w_ceil, cum, yl


def alignment(cum: torch.Tensor, y_lengths: torch.Tensor, t_pad: int, mu: Optional[torch.Tensor],
              want_attn: bool = True):
    """model.py:1283-1289 -> (attn [B,1,Tx,T] | None, mu_y [B,C,T] | None, y_mask [B,1,T])."""
    B, Tx = cum.shape
    dev = cum.device
    attn = torch.empty((B, 1, Tx, t_pad), dtype=torch.float32, device=dev) if want_attn else None
    C = 0 if mu is None else mu.shape[1]
    mu = f32c(mu)
    mu_y = torch.empty((B, C, t_pad), dtype=torch.float32, device=dev) if mu is not None else None
    y_mask = torch.empty((B, 1, t_pad), dtype=torch.float32, device=dev)
    check(lib().mt_alignment(ptr(cum), ptr(y_lengths), B, Tx, t_pad, ptr(mu), C, ptr(attn), ptr(mu_y),
                             ptr(y_mask), stream_handle(dev)), "alignment")
    return attn, mu_y, y_mask


def denorm_crop(z: torch.Tensor, mean: torch.Tensor, std: torch.Tensor, t_y: int) -> torch.Tensor:
    B, C, T = z.shape
    mean = f32c(mean.to(z.device)).reshape(-1).expand(C).contiguous()
    std = f32c(std.to(z.device)).reshape(-1).expand(C).contiguous()
    out = torch.empty((B, C, t_y), dtype=torch.float32, device=z.device)
    check(lib().mt_denorm_crop(ptr(z), ptr(mean), ptr(std), B, C, T, t_y, ptr(out), stream_handle(z.device)),
          "denorm_crop")
    return out


def stft_magnitude(audio: torch.Tensor) -> torch.Tensor:
    require_gpu(audio, what="stft_magnitude")
    audio = f32c(audio)
    B, L = audio.shape
    nfr = 1 + L // 256
    mag = torch.empty((B, nfr, 513), dtype=torch.float32, device=audio.device)
    check(lib().mt_stft_magnitude(ptr(audio), B, L, ptr(mag), stream_handle(audio.device)), "stft_magnitude")
    return mag


def denoise(audio: torch.Tensor, bias_spec: torch.Tensor, strength: float, lengths=None,
            hop: int = 256) -> torch.Tensor:
    """lengths (int [B] in units of `hop` samples, or None): a ragged batch, row b denoised as an utterance of
    hop * lengths[b] samples (mt_denoise_ragged); its output past them is zero"""
    require_gpu(audio, what="denoise")
    audio = f32c(audio)
    B, L = audio.shape
    out = torch.empty((B, 256 * (L // 256)), dtype=torch.float32, device=audio.device)
    bias = f32c(bias_spec.reshape(-1).to(audio.device))
    L_ = lib()
    ws = _Workspace.get(L_.mt_denoise_workspace_bytes(B, L), audio.device)
    if lengths is None:
        check(L_.mt_denoise(ptr(audio), B, L, ptr(bias), float(strength), ptr(out), ws.data_ptr(), ws.numel(),
                            stream_handle(audio.device)), "denoise")
        return out
    lens = lengths.to(device=audio.device, dtype=torch.int32).contiguous()
    if lens.shape != (B,):
        raise ValueError(f"lengths {tuple(lens.shape)}: expected ({B},)")
    check(L_.mt_denoise_ragged(ptr(audio), B, L, ptr(lens), int(hop), ptr(bias), float(strength), ptr(out),
                               ws.data_ptr(), ws.numel(), stream_handle(audio.device)), "denoise")
    return out


def maximum_path(neg_cent: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """train_standalone.py:280-325 on the GPU: neg_cent [B,Tx,Ty], attention mask [B,Tx,Ty] (x_mask x
    y_mask) -> one-hot monotonic path [B,Tx,Ty] in neg_cent's dtype. The lengths are the mask's row /
    column counts at index 0, as the reference takes them."""
    require_gpu(neg_cent, mask, what="maximum_path")
    B, Tx, Ty = neg_cent.shape
    value = f32c(neg_cent.detach())
    t_xs = mask.detach().sum(dim=1)[:, 0].to(torch.int32).contiguous()
    t_ys = mask.detach().sum(dim=2)[:, 0].to(torch.int32).contiguous()
    out = torch.empty((B, Tx, Ty), dtype=torch.float32, device=neg_cent.device)
    L_ = lib()
    ws = _Workspace.get(L_.mt_maximum_path_workspace_bytes(B, Tx, Ty), neg_cent.device)
    check(L_.mt_maximum_path(ptr(value), ptr(t_xs), ptr(t_ys), B, Tx, Ty, ptr(out), ws.data_ptr(), ws.numel(),
                             stream_handle(neg_cent.device)), "maximum_path")
    return out.to(neg_cent.dtype)


def op_conv1d(x_btc: torch.Tensor, W: torch.Tensor, bias: Optional[torch.Tensor], stride=1, pad=0, dil=1,
              transposed=False, slope: Optional[float] = None, precision="fp32", variant: int = -1,
              out: Optional[torch.Tensor] = None, ws: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Op-level test entry: y = conv(lrelu(x)) on [B,T,C] activations (dtype by precision)."""
    require_gpu(x_btc, what="op_conv1d")
    dt = dtype_code(precision)
    et = torch.bfloat16 if dt == DTYPE_BF16 else torch.float32
    x = x_btc.to(et).contiguous()
    B, Tin, cin = x.shape
    if transposed:
        cout, k = W.shape[1], W.shape[2]
        tout = (Tin - 1) * stride - 2 * pad + k
    else:
        cout, k = W.shape[0], W.shape[2]
        tout = (Tin + 2 * pad - dil * (k - 1) - 1) // stride + 1
    y = torch.empty((B, tout, cout), dtype=et, device=x.device) if out is None else out
    L = lib()
    nb = L.mt_op_conv1d_workspace_bytes(dt, cin, cout, k, stride, int(transposed))
    if ws is None or ws.numel() < nb:
        ws = torch.empty(nb, dtype=torch.uint8, device=x.device)
    W, bias = f32c(W), f32c(bias)
    check(L.mt_op_conv1d_tile(int(variant), dt, ptr(x), B, Tin, cin, ptr(W), ptr(bias), cout, k, stride, pad, dil,
                              int(transposed), -1.0 if slope is None else float(slope), ptr(y), tout, ws.data_ptr(),
                              ws.numel(), stream_handle(x.device)), "op_conv1d")
    return y


def op_vconv(x_btc: torch.Tensor, W: torch.Tensor, bias: torch.Tensor, dil: int = 1, ef: int = 0,
             resid: Optional[torch.Tensor] = None, y: Optional[torch.Tensor] = None, y2: Optional[torch.Tensor] = None,
             slope: float = 0.1, div: float = 1.0, ws: Optional[torch.Tensor] = None, pack: bool = True,
             lens: Optional[torch.Tensor] = None):
    """Op-level test entry of mt_vconv: one "same"-padded bf16 Conv1d on an already activated
    [B,L,C] input with the ResBlock epilogues (ef bits: 1 resid, 2 accumulate into y, 4 /div,
    8 y=lrelu(v), 16 also y2=lrelu(v)); lens (int32 [B] on the device): a ragged batch. Returns (y, y2)."""
    require_gpu(x_btc, what="op_vconv")
    x = x_btc.to(torch.bfloat16).contiguous()
    B, L, cin = x.shape
    cout, k = W.shape[0], W.shape[2]
    if y is None:
        y = torch.empty((B, L, cout), dtype=torch.bfloat16, device=x.device)
    if (ef & 16) and y2 is None:
        y2 = torch.empty((B, L, cout), dtype=torch.bfloat16, device=x.device)
    if resid is not None:
        resid = resid.to(torch.bfloat16).contiguous()
    L_ = lib()
    nb = L_.mt_op_vconv_workspace_bytes(cin, cout, k)
    if ws is None or ws.numel() < nb:
        if not pack:
            raise ValueError("op_vconv: pack=False needs the workspace a packing call filled")
        ws = torch.empty(nb, dtype=torch.uint8, device=x.device)
    W, bias = f32c(W), f32c(bias)
    if lens is not None:
        lens = lens.to(device=x.device, dtype=torch.int32).contiguous()
    check(L_.mt_op_vconv(ptr(x), B, L, cin, ptr(W), ptr(bias), cout, k, dil, int(ef), ptr(resid), ptr(y), ptr(y2),
                         float(slope), float(div), ptr(lens), int(bool(pack)), ws.data_ptr(), ws.numel(),
                         stream_handle(x.device)), "op_vconv")
    return y, y2


def set_vconv_ct(enable: bool) -> bool:
    """mt_vconv's compile-time K loop for the decoder's / upsamplers' convs (True, default) or the runtime-cursor
    loop; returns the previous setting (process-wide)"""
    return bool(lib().mt_vconv_set_ct(int(bool(enable))))


def set_vpair_kernels(mask: int) -> int:
    """the round-5 ResBlock pair kernels (bit 0: the 64-channel k = 7 / 11 compile-time K loop; default 1), each
    bit-identical to the kernel it replaces; returns the previous mask (process-wide)"""
    return int(lib().mt_vpair_set_kernels(int(mask)))


def set_post_fold(enable) -> int:
    """conv_post in the last ResBlock pair's epilogue (1, default) or its own launch (0); bit-identical; returns the
    previous setting (process-wide)"""
    return int(lib().mt_vocoder_set_post_fold(int(bool(enable))))


def set_ffn(mode) -> int:
    """the bf16 decoder's transformer FeedForward as one fused launch (mt_ffn; 3, the default: serial schedule with the
    frame fragments prefetched; 1: serial, weight and frame fragments prefetched; 2: FF1 epilogues overlapped with FF2
    steps) or as two mt_vconv GEMMs (False / 0); returns the previous setting (process-wide)"""
    return int(lib().mt_ffn_set(int(mode)))


def set_ffn_min_frames(frames: int) -> int:
    """the fused FeedForward only on decoder levels of at least `frames` frames (B x T; default 16384); returns the
    previous value (process-wide)"""
    return int(lib().mt_ffn_set_min_frames(int(frames)))


def set_decoder_kernels(mask: int) -> int:
    """the decoder kernel variants (bit 0: the dedicated final projection + ODE update kernel; default 1), each
    bit-identical to what it replaces; returns the previous mask (process-wide)"""
    return int(lib().mt_decoder_set_kernels(int(mask)))


def set_rbconv_actin(enable: bool) -> bool:
    """the stage 1-2 ResBlock conv1s activate the raw chain state in LDS (True, default: no activated copies stored)
    or read the activated copies their producers store; returns the previous setting (process-wide)"""
    return bool(lib().mt_vconv_set_actin(int(bool(enable))))


def set_rbconv(enable: bool) -> bool:
    """the HiFi-GAN wide-stage ResBlock convs on mt_rbconv (True, default) or the generic mt_vconv kernel; returns
    the previous setting (process-wide)"""
    return bool(lib().mt_vconv_set_rbconv(int(bool(enable))))


def op_attention(qkv: torch.Tensor, mask: torch.Tensor, heads: int, precision="fp32") -> torch.Tensor:
    require_gpu(qkv, mask, what="op_attention")
    dt = dtype_code(precision)
    et = torch.bfloat16 if dt == DTYPE_BF16 else torch.float32
    qkv = qkv.to(et).contiguous()
    B, T, _ = qkv.shape
    out = torch.empty((B, T, heads * 64), dtype=et, device=qkv.device)
    mask = f32c(mask.reshape(B, T))
    check(lib().mt_op_attention(dt, ptr(qkv), ptr(mask), ptr(out), B, T, heads, stream_handle(qkv.device)),
          "op_attention")
    return out


# ---------------------------------------------------------------------------------- launch probe
PROBE_RBFUSE_C64, PROBE_RBFUSE_C32, PROBE_VCONV, PROBE_VCONV_DEC = 1, 2, 3, 4


def probe_start(site: int, max_launches: int) -> None:
    """Arm HIP events around every launch of one kernel site (see mt_probe_start)."""
    check(lib().mt_probe_start(int(site), int(max_launches)), "probe_start")


def probe_pause(paused: bool) -> None:
    """Stop (True) / resume (False) recording without disarming (see mt_probe_pause)."""
    check(lib().mt_probe_pause(int(bool(paused))), "probe_pause")


PROBE_TAGS = ("vconv", "vpair", "vpair32", "rbfuse", "vpair128", "rbconv")


def probe_detail(cap: int = 4096) -> List[Dict[str, float]]:
    """Per recorded launch (before probe_stop): ms, algorithmic flops / bytes and the kernel kind."""
    from ctypes import c_double
    ms, fl, by, tg = (c_double * cap)(), (c_double * cap)(), (c_double * cap)(), (c_int * cap)()
    n = lib().mt_probe_detail(int(cap), ms, fl, by, tg)
    if n < 0:
        check(n, "probe_detail")
    return [{"ms": ms[i], "flops": fl[i], "bytes": by[i], "kind": PROBE_TAGS[tg[i]]} for i in range(n)]


def probe_stop(peak_flops: float = 2.5e15, peak_bw: float = 8.0e12) -> Dict[str, float]:
    """Synchronize the probe's events: launches, summed kernel ms, algorithmic FLOPs and layer-boundary
    bytes, and the summed per-launch roofline time max(F / peak_flops, B / peak_bw) in ms (defaults: the
    MI355X dense bf16 MFMA and HBM peaks of MI355X_MICROARCH.md)."""
    from ctypes import c_double
    n, ms, fl, by, roof = c_int(0), c_double(0), c_double(0), c_double(0), c_double(0)
    check(lib().mt_probe_stop(byref(n), byref(ms), byref(fl), byref(by), float(peak_flops), float(peak_bw),
                              byref(roof)), "probe_stop")
    return {"launches": n.value, "ms": ms.value, "flops": fl.value, "bytes": by.value, "roof_ms": roof.value}


VCONV_LOG_FIELDS = ("ef", "bm", "bn", "k1", "ntiles", "grid", "taps", "M", "cin", "B", "L")


def vconv_log_start(capacity: int = 65536) -> None:
    """Record the variant and grid of every mt_vconv launch from now on (test coverage)."""
    check(lib().mt_vconv_log_start(int(capacity)), "vconv_log_start")


def vconv_log_stop(capacity: int = 65536) -> List[Dict[str, int]]:
    """Disarm the launch log; one dict per launch (fields VCONV_LOG_FIELDS)."""
    buf = (c_int * (capacity * len(VCONV_LOG_FIELDS)))()
    n = lib().mt_vconv_log_stop(buf, int(capacity))
    k = len(VCONV_LOG_FIELDS)
    return [dict(zip(VCONV_LOG_FIELDS, buf[i * k:(i + 1) * k])) for i in range(n)]
