"""ctypes binding of ``libdotsrl_amd.so`` (the C-ABI declared in ``include/dotsrl_amd.h``).

torch is imported first on purpose: torch ships its own ``libamdhip64.so.7`` and the HIP library is
linked against the same SONAME, so the dynamic loader reuses torch's HIP runtime and both sides share
one device context, one allocator view and the same streams.

There is no fallback: if the library is missing or fails to load, every entry point raises.
"""

from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the HIP library load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DOTSRL_AMD_LIB", os.path.join(_HERE, "libdotsrl_amd.so"))

DRL_I64, DRL_I32, DRL_U8, DRL_F32, DRL_BF16 = 0, 1, 2, 3, 4
DRL_OK = 0
PPO_OUT_N = 8
VALUE_OUT_N = 8

AGG_MODES = {"token-mean": 0, "seq-mean-token-sum": 1, "seq-mean-token-mean": 2, "seq-mean-token-sum-norm": 3}
KL_TYPES = {"kl": 0, "k1": 0, "abs": 1, "mse": 2, "k2": 2, "low_var_kl": 3, "k3": 3}
KL_NONE = -1


class PPOLossParams(ctypes.Structure):
    _fields_ = [
        ("clip_ratio_low", ctypes.c_float),
        ("clip_ratio_high", ctypes.c_float),
        ("clip_ratio_c", ctypes.c_float),
        ("entropy_coeff", ctypes.c_float),
        ("kl_loss_coef", ctypes.c_float),
        ("loss_scale_factor", ctypes.c_float),
        ("loss_agg_mode", ctypes.c_int32),
        ("kl_type", ctypes.c_int32),
        ("token_count", ctypes.c_void_p),
        ("policy_loss", ctypes.c_int32),
        ("cov_ratio", ctypes.c_float),
        ("clip_cov_lb", ctypes.c_float),
        ("clip_cov_ub", ctypes.c_float),
        ("ppo_kl_coef", ctypes.c_float),
        ("cov_seed", ctypes.c_uint64),
    ]


class ValueLossParams(ctypes.Structure):
    _fields_ = [
        ("cliprange_value", ctypes.c_float),
        ("loss_scale_factor", ctypes.c_float),
        ("loss_agg_mode", ctypes.c_int32),
        ("pad", ctypes.c_int32),
    ]


class SamplingParams(ctypes.Structure):
    _fields_ = [
        ("do_sample", ctypes.c_int32),
        ("temperature", ctypes.c_float),
        ("top_k", ctypes.c_int32),
        ("top_p", ctypes.c_float),
        ("seed", ctypes.c_uint64),
        ("offset", ctypes.c_uint64),
        ("row_base", ctypes.c_int64),
        ("pad_token_id", ctypes.c_int64),
        ("eos_ids", ctypes.c_void_p),
        ("n_eos", ctypes.c_int32),
        ("dev_step", ctypes.c_void_p),
    ]


class AdamWParams(ctypes.Structure):
    _fields_ = [
        ("lr", ctypes.c_float),
        ("beta1", ctypes.c_float),
        ("beta2", ctypes.c_float),
        ("eps", ctypes.c_float),
        ("weight_decay", ctypes.c_float),
        ("step", ctypes.c_int32),
        ("max_grad_norm", ctypes.c_float),
    ]


P = ctypes.c_void_p
I64 = ctypes.c_int64
I32 = ctypes.c_int32
F32 = ctypes.c_float
SZ = ctypes.c_size_t

# name -> (restype, argtypes); must match include/dotsrl_amd.h exactly
ABI_VERSION = 8  # include/dotsrl_amd.h DRL_ABI_VERSION: the layouts below (PPOLossParams) are of this version

SIGNATURES = {
    "drl_last_error": (ctypes.c_char_p, []),
    "drl_abi_version": (ctypes.c_int, []),
    "drl_device_cu_count": (ctypes.c_int, []),
    "drl_ppo_loss_workspace_bytes": (SZ, [I64, I64]),
    "drl_ppo_loss_fwd_bwd": (ctypes.c_int, [P, P, P, P, I32, P, P, I64, I64, ctypes.POINTER(PPOLossParams), P, P, P, P,
                                            SZ, P]),
    "drl_kl_penalty": (ctypes.c_int, [P, P, I64, I32, P, P]),
    "drl_agg_loss_workspace_bytes": (SZ, [I64, I64]),
    "drl_agg_loss": (ctypes.c_int, [P, P, I32, I64, I64, I32, P, P, SZ, P]),
    "drl_logprob_entropy_fwd": (ctypes.c_int, [P, I32, I64, I64, I64, P, F32, P, P, P, P]),
    "drl_token_logprob": (ctypes.c_int, [P, I32, I64, I64, I64, P, I64, P, F32, P, I64, P]),
    "drl_logprob_entropy_bwd": (ctypes.c_int, [P, I32, I64, I64, I64, P, F32, P, P, P, P, P, I32, I64, P]),
    "drl_grpo_workspace_bytes": (SZ, [I64]),
    "drl_grpo_outcome_advantage": (ctypes.c_int, [P, P, I32, P, P, P, I64, I64, I64, F32, I32, P, P, P, SZ, P]),
    "drl_group_outcome_advantage_workspace_bytes": (SZ, [I64]),
    "drl_group_outcome_advantage": (ctypes.c_int, [P, P, I32, P, P, P, I64, I64, I64, I32, F32, I32, P, P, P, SZ, P]),
    "drl_reinforce_pp_advantage_return": (ctypes.c_int, [P, P, I32, I64, I64, F32, P, P, P, SZ, P]),
    "drl_remax_advantage_return": (ctypes.c_int, [P, P, P, I32, I64, I64, P, P, P]),
    "drl_decode_step_prologue_workspace_bytes": (SZ, []),
    "drl_decode_step_prologue": (ctypes.c_int, [P, I64, P, P, P, I64, P, I32, I64, I64, I64, P, P, P, P, I64, P, SZ, I64,
                                                P]),
    "drl_gae_workspace_bytes": (SZ, [I64, I64]),
    "drl_gae_advantage_return": (ctypes.c_int, [P, P, I32, P, I32, I64, I64, F32, F32, P, P, P, SZ, P]),
    "drl_value_loss_workspace_bytes": (SZ, [I64, I64]),
    "drl_value_loss_fwd_bwd": (ctypes.c_int, [P, P, I32, P, P, I32, I64, I64, ctypes.POINTER(ValueLossParams), P, P, P,
                                              SZ, P]),
    "drl_value_head_fwd": (ctypes.c_int, [P, I64, P, P, I32, I64, I64, P, I32, P]),
    "drl_value_head_bwd_workspace_bytes": (SZ, [I64, I64]),
    "drl_value_head_bwd": (ctypes.c_int, [P, I64, P, I32, P, I64, I64, P, I64, P, P, P, SZ, P]),
    "drl_select_tokens_workspace_bytes": (SZ, [I64, I64]),
    "drl_select_tokens": (ctypes.c_int, [P, I32, I64, I64, I64, ctypes.POINTER(SamplingParams), P, P, I64, P, SZ, P]),
    "drl_response_mask": (ctypes.c_int, [P, I64, I64, I64, P, I32, P, I32, I64, P]),
    "drl_position_ids": (ctypes.c_int, [P, I32, I64, I64, P, P]),
    "drl_response_position_ids": (ctypes.c_int, [P, I64, I64, I64, P]),
    "drl_grad_norm_workspace_bytes": (SZ, [I64]),
    "drl_grad_norm": (ctypes.c_int, [P, I64, P, P, SZ, P]),
    "drl_adamw_step": (ctypes.c_int, [P, P, P, P, P, I64, ctypes.POINTER(AdamWParams), P, P]),
    "drl_rope_qkv_fwd": (ctypes.c_int, [P, I32, P, P, P, I64, I64, I64, I64, I64, I64, P, P, P, I64, I64, P, P, P, P,
                                        I64, P]),
    "drl_rope_qkv_fwd_rows": (ctypes.c_int, [P, P, I32, P, P, P, I64, I64, I64, I64, I64, I64, P, P, P, I64, I64, P, P,
                                             P, P, I64, P, P]),
    "drl_rope_qkv_bwd": (ctypes.c_int, [P, P, P, I32, P, P, P, I64, I64, I64, I64, I64, I64, P, P]),
    "drl_masked_softmax_fwd": (ctypes.c_int, [P, P, I32, P, I64, I64, I64, I64, I64, I64, F32, P]),
    "drl_masked_softmax_bwd": (ctypes.c_int, [P, P, P, I32, I64, I64, F32, P]),
    "drl_add_rmsnorm_fwd": (ctypes.c_int, [P, P, P, P, P, I32, P, I64, I64, F32, P]),
    "drl_rmsnorm_bwd_workspace_bytes": (SZ, [I64, I64]),
    "drl_rmsnorm_bwd": (ctypes.c_int, [P, P, P, P, I32, P, P, I64, I64, P, SZ, P]),
    "drl_rmsnorm_bwd_ex": (ctypes.c_int, [P, P, P, P, I32, P, P, P, P, I64, I64, P, SZ, P]),
    "drl_swiglu_fwd": (ctypes.c_int, [P, P, I32, I64, I64, P]),
    "drl_swiglu_bwd": (ctypes.c_int, [P, P, P, I32, I64, I64, P]),
    "drl_decode_attention_workspace_bytes": (SZ, [I64, I64, I64, I64, I64]),
    "drl_flash_attn_fwd": (ctypes.c_int, [P, P, P, I32, P, I64, I64, I64, I64, I64, I64, I64, I64, I64, I64, P, F32,
                                          P, P, P]),
    "drl_flash_attn_fwd_rows": (ctypes.c_int, [P, P, P, I32, P, I64, I64, I64, I64, I64, I64, I64, I64, I64, I64, P,
                                               F32, P, P, P, P]),
    "drl_decode_attention_vt_workspace_bytes": (SZ, [I64, I64, I64, I64]),
    "drl_decode_attention_set_plan": (None, [I32, I32]),
    "drl_decode_group_set_plan": (None, [I32, I32, I32]),
    "drl_flash_attn_bwd_set_variant": (None, [I32]),
    "drl_decode_attention_vt": (ctypes.c_int, [P, P, P, I32, P, I64, P, I64, I64, I64, I64, I64, I64, I64, I64, I64,
                                               I64, F32, P, I64, P, SZ, P]),
    "drl_flash_attn_bwd": (ctypes.c_int, [P, P, P, P, P, P, P, I32, P, I64, I64, I64, I64, I64, I64, I64, P, F32, P, P, P,
                                          P, P]),
    "drl_flash_attn_bwd_rows": (ctypes.c_int, [P, P, P, P, P, P, P, P, I32, P, I64, I64, I64, I64, I64, I64, I64, P,
                                               F32, P, P, P, P, P]),
    "drl_decode_attention": (ctypes.c_int, [P, P, P, I32, P, I64, P, I64, I64, I64, I64, I64, I64, I64, F32, P, P, SZ,
                                            P]),
    "drl_linear_logprob_workspace_bytes": (SZ, [I64, I64, I64]),
    "drl_linear_select_tokens_workspace_bytes": (SZ, [I64]),
    "drl_linear_select_tokens": (ctypes.c_int, [P, I64, P, I32, I64, I64, I64, P, P, P, I64, P, SZ, P]),
    "drl_decode_attention_set_variant": (None, [I32]),
    "drl_decode_gemm_plan": (ctypes.c_int, [I64, I64, I64, I32, P, P]),
    "drl_decode_gemm_set_plan": (None, [I32, I32]),
    "drl_decode_gemm_set_tiled": (None, [I32]),
    "drl_decode_gemm_set_max_splits": (None, [I32]),
    "drl_gemm": (ctypes.c_int, [P, I64, I32, P, I64, I32, P, I64, I32, I32, I64, I64, I64, P, I32, P, I64, P, I64, P]),
    "drl_gemm_workspace_bytes": (ctypes.c_int64, []),
    "drl_gemm_set_sk_tuning": (None, [I32, I32, I32, I32]),
    "drl_gemm_set_debug": (None, [I32]),
    "drl_gemm_plan": (ctypes.c_int, [I64, I64, I64, I32, I32, P]),
    "drl_copy_rows": (ctypes.c_int, [P, I64, P, P, I64, P, I64, I64, P]),
    "drl_gather_rows": (ctypes.c_int, [P, I64, P, P, I64, I64, I64, P]),
    "drl_sum_rows": (ctypes.c_int, [P, I64, P, I64, P, I64, P, I64, I64, I32, P]),
    "drl_colsum_bf16_workspace_bytes": (SZ, [I64, I64]),
    "drl_colsum_bf16_acc": (ctypes.c_int, [P, I64, I64, I64, P, P, SZ, P]),
    "drl_decode_gemm_force_tiled": (None, [I32, I32]),
    "drl_decode_pack_weight_elems": (SZ, [I64, I64, I32]),
    "drl_decode_pack_weight": (ctypes.c_int, [P, I64, I64, I64, I32, P, P]),
    "drl_decode_gemm": (ctypes.c_int, [P, P, I64, I64, I64, I32, P, P, P]),
    "drl_decode_rmsnorm": (ctypes.c_int, [P, P, I32, P, P, P, I64, I64, I64, F32, P, I64, P]),
    "drl_decode_pack_weight_rope": (ctypes.c_int, [P, I64, I64, I64, I64, P, P]),
    "drl_decode_qkv_rope": (ctypes.c_int, [P, P, P, P, P, P, I64, I64, I64, I64, I64, I64, P, P, P, I64, I64, P, P]),
    "drl_decode_rope": (ctypes.c_int, [P, I32, P, P, P, P, I64, I64, I64, I64, I64, P, P, P, P, I64, I64, I64, P, P]),
    "drl_decode_norm_plan": (ctypes.c_int, [I64, I64, I64, I32, P, P, P]),
    "drl_decode_norm_set_plan": (None, [I32, I32, I32]),
    "drl_decode_resid_counter_bytes": (SZ, [I64, I64, I64]),
    "drl_decode_gemm_resid": (ctypes.c_int, [P, P, I64, I64, I64, P, I64, P, P, SZ, P]),
    "drl_decode_gemm_norm": (ctypes.c_int, [P, P, F32, P, I64, I64, I64, P, P]),
    "drl_decode_qkv_rope_norm": (ctypes.c_int, [P, P, F32, P, P, P, P, P, I64, I64, I64, I64, I64, I64, P, P, P, I64,
                                                I64, P, P]),
    "drl_decode_final_norm": (ctypes.c_int, [P, I64, P, P, I64, I64, I64, F32, P, I64, P]),
    "drl_decode_lm_head_plan": (ctypes.c_int, [I64, I64, I64, P]),
    "drl_decode_lm_head_set_config": (None, [I32]),
    "drl_decode_lm_head": (ctypes.c_int, [P, I64, P, I64, I64, I64, P, I64, P]),
    "drl_linear_logprob_fwd": (ctypes.c_int, [P, I64, P, P, I32, I64, I64, I64, F32, P, P, P, P, SZ, P]),
    "drl_linear_logprob_dlogits": (ctypes.c_int, [P, I64, P, P, I32, I64, I64, I64, F32, P, P, P, P, P, I64, P]),
}

_lib = None
_lock = threading.Lock()


class NativeLibraryError(RuntimeError):
    pass


def load(path: str | None = None):
    """Load (once) and return the ctypes handle; raises NativeLibraryError if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        # DRL_LIB_PATH: an alternative build of the same ABI (A/B kernel measurements, tools/gemm_sk_bench.py)
        p = path or os.environ.get("DRL_LIB_PATH") or LIB_PATH
        if not os.path.exists(p):
            raise NativeLibraryError(
                f"HIP library not found at {p}: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "or `make -C dots.rl_amd/csrc` (there is no CPU/eager fallback)")
        lib = ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.drl_abi_version() != ABI_VERSION:
            raise NativeLibraryError(f"ABI mismatch: library reports {lib.drl_abi_version()}")
        _lib = lib
    return _lib


def check(rc: int, what: str = ""):
    if rc != DRL_OK:
        msg = load().drl_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (code {rc}): {msg}")
