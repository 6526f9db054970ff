"""ctypes binding of libmatcha_hip.so (C ABI: include/matcha_hip.h).

The library is built in-tree (``make -C matcha-tts_amd`` or ``__graft_entry__.build()``)
and loaded from ``matcha-tts_amd/libmatcha_hip.so``. There is no fallback: if the
library is missing, every HIP entry point raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_float, c_int, c_int64, c_size_t, c_uint, c_void_p

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(PKG_DIR, "libmatcha_hip.so")

DTYPE_F32 = 0
DTYPE_BF16 = 1
SOLVER_EULER = 0
SOLVER_MIDPOINT = 1

P = c_void_p  # device pointer / opaque handle

# name -> (restype, argtypes); mirrors include/matcha_hip.h one to one
SIGNATURES = {
    "mt_last_error": (c_char_p, []),
    "mt_abi_version": (c_int, []),
    "mt_build_experiments": (c_int, []),
    "mt_sched_count": (c_int, []),
    "mt_sched_get": (c_int, [c_int, P, P, P, c_int]),
    "mt_encoder_create": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                  POINTER(c_void_p)]),
    "mt_encoder_destroy": (None, [P]),
    "mt_encoder_num_params": (c_int, [P]),
    "mt_encoder_param_name": (c_int, [P, c_int, c_char_p, c_int]),
    "mt_encoder_param_shape": (c_int, [P, c_int, POINTER(c_int64), c_int]),
    "mt_encoder_packed_bytes": (c_size_t, [P]),
    "mt_encoder_pack": (c_int, [P, POINTER(c_void_p), P, P]),
    "mt_encoder_workspace_bytes": (c_size_t, [P, c_int, c_int]),
    "mt_encoder_set_mfma_attention": (c_int, [P, c_int]),
    "mt_encoder_set_vconv": (c_int, [P, c_int]),
    "mt_encoder_set_split": (c_int, [P, c_int]),
    "mt_encoder_forward": (c_int, [P, P, P, P, P, c_int, c_int, P, P, P, P, P, c_size_t, P]),
    "mt_decoder_create": (c_int, [c_int, c_int, c_int, c_int, c_int, POINTER(c_void_p)]),
    "mt_decoder_destroy": (None, [P]),
    "mt_decoder_num_params": (c_int, [P]),
    "mt_decoder_param_name": (c_int, [P, c_int, c_char_p, c_int]),
    "mt_decoder_param_shape": (c_int, [P, c_int, POINTER(c_int64), c_int]),
    "mt_decoder_packed_bytes": (c_size_t, [P]),
    "mt_decoder_pack": (c_int, [P, POINTER(c_void_p), P, P]),
    "mt_cfm_workspace_bytes": (c_size_t, [P, c_int, c_int, c_int, c_int]),
    "mt_cfm_solve": (c_int, [P, P, P, c_float, P, P, P, c_int, c_int, c_int, c_int, P, P, c_size_t, P]),
    "mt_cfm_solve_bounded": (c_int, [P, P, P, c_float, P, P, P, c_int, c_int, c_int, c_int, c_int, P, P, c_size_t,
                                     P]),
    "mt_decoder_set_uniform_attention": (c_int, [P, c_int]),
    "mt_decoder_set_graphs": (c_int, [P, c_int]),
    "mt_decoder_set_taps": (c_int, [P, P, c_int]),
    "mt_decoder_step_workspace_bytes": (c_size_t, [P, c_int, c_int]),
    "mt_decoder_step": (c_int, [P, P, P, P, P, P, c_float, c_int, c_int, P, P, c_size_t, P]),
    "mt_vocoder_create": (c_int, [c_int, c_int, POINTER(c_int), POINTER(c_int), c_int, c_int,
                                  POINTER(c_int), c_int, POINTER(c_int), c_int, POINTER(c_void_p)]),
    "mt_vocoder_destroy": (None, [P]),
    "mt_vocoder_num_params": (c_int, [P]),
    "mt_vocoder_param_name": (c_int, [P, c_int, c_char_p, c_int]),
    "mt_vocoder_param_shape": (c_int, [P, c_int, POINTER(c_int64), c_int]),
    "mt_vocoder_packed_bytes": (c_size_t, [P]),
    "mt_vocoder_set_fusion": (c_int, [P, c_int]),
    "mt_vocoder_set_vconv": (c_int, [P, c_int]),
    "mt_vocoder_set_pair": (c_int, [P, c_int]),
    "mt_decoder_set_vconv": (c_int, [P, c_int]),
    "mt_vocoder_pack": (c_int, [P, POINTER(c_void_p), P, P]),
    "mt_vocoder_workspace_bytes": (c_size_t, [P, c_int, c_int]),
    "mt_vocoder_forward": (c_int, [P, P, P, c_int, c_int, P, P, c_size_t, P]),
    "mt_vocoder_forward_ragged": (c_int, [P, P, P, c_int, c_int, P, P, P, c_size_t, P]),
    "mt_vocoder_ragged_supported": (c_int, [P]),
    "mt_durations": (c_int, [P, P, c_float, c_int, c_int, P, P, P, P]),
    "mt_alignment": (c_int, [P, P, c_int, c_int, c_int, P, c_int, P, P, P, P]),
    "mt_denorm_crop": (c_int, [P, P, P, c_int, c_int, c_int, c_int, P, P]),
    "mt_denoise_workspace_bytes": (c_size_t, [c_int, c_int]),
    "mt_denoise": (c_int, [P, c_int, c_int, P, c_float, P, P, c_size_t, P]),
    "mt_denoise_ragged": (c_int, [P, c_int, c_int, P, c_int, P, c_float, P, P, c_size_t, P]),
    "mt_maximum_path_workspace_bytes": (c_size_t, [c_int, c_int, c_int]),
    "mt_decoder_step_times_workspace_bytes": (c_size_t, [P, c_int, c_int]),
    "mt_decoder_step_times": (c_int, [P, P, P, P, P, P, P, c_int, c_int, P, P, c_size_t, P]),
    "mt_maximum_path": (c_int, [P, P, P, c_int, c_int, c_int, P, P, c_size_t, P]),
    "mt_stft_magnitude": (c_int, [P, c_int, c_int, P, P]),
    "mt_log_mel": (c_int, [P, c_int, c_int, P, c_float, c_float, P, P]),
    "mt_op_conv1d_workspace_bytes": (c_size_t, [c_int, c_int, c_int, c_int, c_int, c_int]),
    "mt_op_conv1d": (c_int, [c_int, P, c_int, c_int, c_int, P, P, c_int, c_int, c_int, c_int, c_int,
                             c_int, c_float, P, c_int, P, c_size_t, P]),
    "mt_op_conv1d_tile": (c_int, [c_int, c_int, P, c_int, c_int, c_int, P, P, c_int, c_int, c_int, c_int, c_int,
                                  c_int, c_float, P, c_int, P, c_size_t, P]),
    "mt_op_vconv_workspace_bytes": (c_size_t, [c_int, c_int, c_int]),
    "mt_op_vconv": (c_int, [P, c_int, c_int, c_int, P, P, c_int, c_int, c_int, c_int, P, P, P, c_float, c_float,
                            P, c_int, P, c_size_t, P]),
    "mt_vconv_set_rbconv": (c_int, [c_int]),
    "mt_vconv_set_ct": (c_int, [c_int]),
    "mt_vpair_set_kernels": (c_int, [c_int]),
    "mt_vocoder_set_post_fold": (c_int, [c_int]),
    "mt_ffn_set": (c_int, [c_int]),
    "mt_vconv_set_actin": (c_int, [c_int]),
    "mt_ffn_set_min_frames": (c_int, [c_int]),
    "mt_decoder_set_kernels": (c_int, [c_int]),
    "mt_op_attention": (c_int, [c_int, P, P, P, c_int, c_int, c_int, P]),
    "mt_probe_start": (c_int, [c_int, c_int]),
    "mt_probe_pause": (c_int, [c_int]),
    "mt_probe_detail": (c_int, [c_int, P, P, P, P]),
    "mt_probe_stop": (c_int, [P, P, P, P, c_double, c_double, P]),
    "mtt_gemm": (c_int, [c_int, c_int, c_int, c_int, c_int, c_float, P, c_int, c_int64, P, c_int, c_int64, c_float,
                         P, c_int, c_int64, c_int, P, P, P, c_size_t, P]),
    "mtt_gemm_ex": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_float, P, c_int, c_int64, P, c_int, c_int64,
                            c_float, P, c_int, c_int64, c_int, P, P, P, c_size_t, P]),
    "mtt_gemm_workspace_bytes": (c_size_t, [c_int, c_int, c_int, c_int]),
    "mtt_im2col": (c_int, [P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, P, P]),
    "mtt_col2im": (c_int, [P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, P, c_int, P]),
    "mtt_ew": (c_int, [c_int, c_size_t, P, P, P, P, c_float, c_float, c_size_t, c_size_t, c_size_t, c_size_t,
                       c_size_t, c_size_t, c_int, P]),
    "mtt_copy_cols": (c_int, [P, c_int, c_int, P, c_int, c_int, c_int, c_int, c_int, P]),
    "mtt_seq_mask": (c_int, [P, c_int, c_int, P, P]),
    "mtt_colsum_scratch_floats": (c_size_t, [c_int, c_int, c_int]),
    "mtt_colsum": (c_int, [P, P, c_int, c_int, c_int, P, c_int, P, P]),
    "mtt_sum": (c_int, [P, P, c_size_t, P, P, P]),
    "mtt_dropout": (c_int, [P, c_size_t, c_float, c_uint, P, P]),
    "mtt_groupnorm_fwd": (c_int, [P, P, P, c_int, c_int, c_int, c_int, c_float, P, P, P, P]),
    "mtt_groupnorm_bwd": (c_int, [P, P, P, P, P, c_int, c_int, c_int, c_int, P, P, P, P]),
    "mtt_layernorm_fwd": (c_int, [P, P, P, c_int, c_int, c_float, P, P, P, P]),
    "mtt_layernorm_bwd": (c_int, [P, P, P, P, P, c_int, c_int, P, P]),
    "mtt_snake_fwd": (c_int, [P, P, P, c_size_t, c_int, P, P]),
    "mtt_snake_bwd": (c_int, [P, P, P, P, c_size_t, c_int, P, P, P, P]),
    "mtt_softmax_fwd": (c_int, [P, P, P, c_int, c_int, c_int, c_int, c_float, c_int, P, P]),
    "mtt_softmax_bwd": (c_int, [P, P, P, P, c_int, c_int, c_int, c_int, c_float, P, P]),
    "mtt_rope": (c_int, [P, c_int, c_int, c_int, c_int, c_int, P, c_int, P]),
    "mtt_embed_fwd": (c_int, [P, c_size_t, P, c_int, c_float, P, P]),
    "mtt_embed_bwd": (c_int, [P, c_size_t, P, c_int, c_int, c_float, P, P]),
    "mtt_adam": (c_int, [P, P, P, P, c_size_t, P, c_float, c_float, c_float, c_float, c_int, P]),
    "mtt_clip_factor": (c_int, [P, c_float, c_float, P, P, P]),
    "mtt_unscale": (c_int, [P, c_size_t, c_float, P, P, P]),
    "mt_vconv_log_start": (c_int, [c_int]),
    "mt_vconv_log_stop": (c_int, [P, c_int]),
}

_lib = None


class HipPathError(RuntimeError):
    """Raised when the native library is unavailable or a C entry point fails."""


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise HipPathError(
                f"{LIB_PATH} is missing: build it with `make -C matcha-tts_amd` "
                "(or __graft_entry__.build()); there is no CPU fallback")
        L = ctypes.CDLL(LIB_PATH)
        # timing experiments against an OLDER build of the library (tools/*: MT_LIB) may lack newer entry points
        older = os.environ.get("MT_LIB") is not None and os.path.abspath(LIB_PATH) == os.path.abspath(
            os.environ["MT_LIB"])
        for name, (res, args) in SIGNATURES.items():
            if older and not hasattr(L, name):
                continue
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        # a timing-experiment build (tools/exp_build.sh) drops kernel work and computes wrong results: only the
        # timing tools may load one, explicitly through MT_LIB
        if not older and hasattr(L, "mt_build_experiments") and L.mt_build_experiments() != 0:
            raise HipPathError(
                f"{LIB_PATH} is a timing-experiment build (mt_build_experiments() = {L.mt_build_experiments():#x}): "
                "rebuild it with `make -C matcha-tts_amd`")
        _lib = L
    return _lib


def build_experiments() -> int:
    """Experiment macros the loaded library was built with (include/matcha_hip.h mt_build_experiments; 0 =
    production build)."""
    return int(lib().mt_build_experiments())


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().mt_last_error().decode(errors="replace")
        raise HipPathError(f"matcha_hip {what} failed ({rc}): {msg}")


def ptr(t) -> int:
    """Device pointer of a tensor (None -> NULL)."""
    return None if t is None else t.data_ptr()


def stream_handle(device=None) -> int:
    import torch
    return torch.cuda.current_stream(device).cuda_stream
