"""Torch-facing wrappers over the C-ABI (device pointers + the current HIP stream, nothing else).

PyTorch-ROCm provides storage, streams and the allocator; every arithmetic step of the hot path runs
in the gfx950 kernels of ``libdotsrl_amd.so``. Tensors must live on the GPU; anything else raises.
"""

from __future__ import annotations

import ctypes
import functools
import math
import threading

import torch

from . import _lib
from ._lib import check

_MASK_DTYPES = {torch.int64: _lib.DRL_I64, torch.int32: _lib.DRL_I32, torch.uint8: _lib.DRL_U8,
                torch.bool: _lib.DRL_U8, torch.float32: _lib.DRL_F32}
_LOGIT_DTYPES = {torch.float32: _lib.DRL_F32, torch.bfloat16: _lib.DRL_BF16}


def lib():
    L = _lib.load()
    return _TimedLib(L) if _TIMERS else L


# ----------------------------------------------------------------------------------------------- timing
_TIMERS: dict = {}


class KernelTimer:
    """Brackets every launch of one C-ABI entry point with HIP events on the stream it is launched on
    (the current torch stream, which every wrapper passes to the library) while active; launches recorded
    into a HIP graph are not timed. ``bytes_fn(args)`` gives the algorithmic bytes of one launch from the
    entry point's own arguments. Used by bench.py for the roofline of the dominant kernel."""

    def __init__(self, symbol: str, bytes_fn, tag_fn=None):
        self.symbol, self.bytes_fn, self.tag_fn = symbol, bytes_fn, tag_fn
        self.events, self.nbytes, self.tags, self.streams = [], [], [], []

    def __enter__(self):
        _TIMERS[self.symbol] = self
        return self

    def __exit__(self, *exc):
        _TIMERS.pop(self.symbol, None)

    def wrap(self, fn):
        def call(*args):
            if torch.cuda.is_current_stream_capturing():
                return fn(*args)
            s = torch.cuda.current_stream()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            rc = fn(*args)
            b.record(s)
            self.events.append((a, b))
            self.nbytes.append(self.bytes_fn(args))
            self.streams.append(s.cuda_stream)
            if self.tag_fn is not None:
                self.tags.append(self.tag_fn(args))
            return rc
        return call

    def summary(self):
        """(launches, mean seconds per launch, mean algorithmic bytes per launch)."""
        if not self.events:
            return 0, float("nan"), float("nan")
        torch.cuda.synchronize()
        tot = sum(a.elapsed_time(b) for a, b in self.events) * 1e-3
        n = len(self.events)
        return n, tot / n, sum(self.nbytes) / n

    def intervals(self):
        """Per launch: (start_us, end_us) relative to the first launch's start, the stream handle, the algorithmic
        work and the tag (``tag_fn(args)``, e.g. the GEMM shape)."""
        if not self.events:
            return []
        torch.cuda.synchronize()
        t0 = self.events[0][0]
        out = []
        for i, (a, b) in enumerate(self.events):
            out.append((t0.elapsed_time(a) * 1e3, t0.elapsed_time(b) * 1e3, self.streams[i], self.nbytes[i],
                        self.tags[i] if self.tags else None))
        return out

    def busy_seconds(self):
        """Length of the union of the launch intervals: launches on two streams (a weight gradient beside its input
        gradient) overlap, and each one's own interval then includes the time it shared the CUs."""
        if not self.events:
            return float("nan")
        torch.cuda.synchronize()
        t0 = self.events[0][0]
        iv = sorted((t0.elapsed_time(a), t0.elapsed_time(b)) for a, b in self.events)
        busy, cur_s, cur_e = 0.0, iv[0][0], iv[0][1]
        for s_, e_ in iv[1:]:
            if s_ > cur_e:
                busy += cur_e - cur_s
                cur_s, cur_e = s_, e_
            else:
                cur_e = max(cur_e, e_)
        return (busy + cur_e - cur_s) * 1e-3


class _TimedLib:
    def __init__(self, real):
        self._real = real

    def __getattr__(self, name):
        fn = getattr(self._real, name)
        t = _TIMERS.get(name)
        return fn if t is None else t.wrap(fn)


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


# Workspace lane: the graphed decode step can run independent row groups ("lanes") of one rollout on separate
# streams inside one graph (rollout.MI355XRollout._decode_graphed). Every stateful workspace (zero-state flag /
# ticket words, the selection scratch, drl_gemm's stream-K slabs) is keyed by the lane, so concurrent lanes never
# share one; lane 0 is the default everywhere else.
# The lane is thread-local: concurrent passes issued from two host threads (trainer: old and ref log-probs) each
# carry their own.
class _LaneState(threading.local):
    lane = 0


_LANE_STATE = _LaneState()


def _lane():
    return _LANE_STATE.lane


class workspace_lane:
    """Context manager: calls inside (on this host thread) use lane ``j``'s workspaces."""

    def __init__(self, j):
        self.j = int(j)

    def __enter__(self):
        self.prev = _LANE_STATE.lane
        _LANE_STATE.lane = self.j
        return self

    def __exit__(self, *exc):
        _LANE_STATE.lane = self.prev
        return False


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _dev(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise ValueError("dots.rl_amd kernels take GPU tensors (there is no CPU path)")


def _c(t):
    return None if t is None else t.contiguous()


def _c16(t):
    """Contiguous with a 16-byte aligned base (the vectorised kernels' requirement): a row slice of a larger
    batch (e.g. a micro-batch of one sequence) is copied once into a fresh allocation."""
    if t is None:
        return None
    t = t.contiguous()
    return t if t.data_ptr() % 16 == 0 else t.clone()


class _Workspace:
    """Per-device scratch buffer, grown on demand; stream-ordered reuse on the current stream."""

    def __init__(self):
        self.buf = {}

    def get(self, nbytes: int, device) -> torch.Tensor:
        key = (device.index if device.index is not None else torch.cuda.current_device(), _lane())
        b = self.buf.get(key)
        if b is None or b.numel() < nbytes:
            b = torch.empty(max(nbytes, 1 << 16), dtype=torch.uint8, device=device)
            self.buf[key] = b
        return b


_ws = _Workspace()


class _ZeroHeaderWorkspace(_Workspace):
    """K1's scratch: zeroed at allocation; the kernel leaves its 256-byte header zero after every call
    (include/dotsrl_amd.h, drl_ppo_loss_fwd_bwd), so no per-call memset."""

    def get(self, nbytes: int, device) -> torch.Tensor:
        key = (device.index if device.index is not None else torch.cuda.current_device(), _lane())
        b = self.buf.get(key)
        if b is None or b.numel() < nbytes:
            b = torch.zeros(max(nbytes, 1 << 16), dtype=torch.uint8, device=device)
            self.buf[key] = b
        return b


_ws_k1 = _ZeroHeaderWorkspace()


def mask_dtype_code(mask: torch.Tensor) -> int:
    try:
        return _MASK_DTYPES[mask.dtype]
    except KeyError as e:
        raise ValueError(f"unsupported mask dtype {mask.dtype}") from e


# ----------------------------------------------------------------------------------------------- K1
def ppo_loss_fwd_bwd(old_log_prob, log_prob, advantages, response_mask, entropy=None, ref_log_prob=None, *,
                     clip_ratio_low=0.2, clip_ratio_high=0.2, clip_ratio_c=3.0, entropy_coeff=0.0,
                     kl_loss_coef=0.0, kl_loss_type=None, loss_agg_mode="token-mean", loss_scale_factor=1.0,
                     want_dlogp=True, want_dentropy=False, out=None, dlogp=None, dentropy=None, token_count=None,
                     policy_loss="vanilla", cov_ratio=0.0002, clip_cov_lb=1.0, clip_cov_ub=5.0, ppo_kl_coef=0.1,
                     cov_seed=0):
    """One launch: the 8 loss scalars (see DRL_PPO_OUT_*) and d loss / d log_prob, d loss / d entropy.
    ``token_count`` (token-mean): device float64 scalar = response_mask.sum() when the caller already has
    it; K1 then makes one pass over HBM instead of two."""
    _dev(old_log_prob, log_prob, advantages, response_mask, entropy, ref_log_prob)
    old_log_prob, log_prob, advantages = _c16(old_log_prob.float()), _c16(log_prob.float()), _c16(advantages.float())
    response_mask = _c16(response_mask)
    entropy = _c16(entropy.float()) if entropy is not None else None
    ref_log_prob = _c16(ref_log_prob.float()) if ref_log_prob is not None else None
    B, R = log_prob.shape
    prm = _lib.PPOLossParams(clip_ratio_low, clip_ratio_high, clip_ratio_c, entropy_coeff, kl_loss_coef,
                             loss_scale_factor, _lib.AGG_MODES[loss_agg_mode],
                             _lib.KL_NONE if kl_loss_type is None else _lib.KL_TYPES[kl_loss_type], None,
                             {"vanilla": 0, "gpg": 1, "gspo": 2, "geo_mean": 3, "clip_cov": 4, "kl_cov": 5}[policy_loss],
                             float(cov_ratio), float(clip_cov_lb), float(clip_cov_ub), float(ppo_kl_coef),
                             int(cov_seed) & 0xFFFFFFFFFFFFFFFF)
    if token_count is not None:
        _dev(token_count)
        assert token_count.dtype == torch.float64 and token_count.numel() == 1
        prm.token_count = token_count.data_ptr()
    dev = log_prob.device
    if out is None:
        out = torch.empty(_lib.PPO_OUT_N, dtype=torch.float32, device=dev)
    if want_dlogp and dlogp is None:
        dlogp = torch.empty_like(log_prob)
    if want_dentropy and dentropy is None:
        dentropy = torch.empty_like(log_prob)
    L = lib()
    nb = L.drl_ppo_loss_workspace_bytes(B, R)
    ws = _ws_k1.get(nb, dev)
    check(L.drl_ppo_loss_fwd_bwd(_p(old_log_prob), _p(log_prob), _p(advantages), _p(response_mask),
                                 mask_dtype_code(response_mask), _p(entropy), _p(ref_log_prob), B, R,
                                 ctypes.byref(prm), _p(out), _p(dlogp if want_dlogp else None),
                                 _p(dentropy if want_dentropy else None), _p(ws), ws.numel(), _stream()),
          "drl_ppo_loss_fwd_bwd")
    return out, (dlogp if want_dlogp else None), (dentropy if want_dentropy else None)


def kl_penalty(log_prob, ref_log_prob, kl_type: str):
    _dev(log_prob, ref_log_prob)
    a, b = _c(log_prob.float()), _c(ref_log_prob.float())
    out = torch.empty_like(a)
    check(lib().drl_kl_penalty(_p(a), _p(b), a.numel(), _lib.KL_TYPES[kl_type], _p(out), _stream()), "drl_kl_penalty")
    return out


def agg_loss(loss_mat, loss_mask, loss_agg_mode):
    _dev(loss_mat, loss_mask)
    x, m = _c(loss_mat.float()), _c(loss_mask)
    B, R = x.shape
    out = torch.empty((), dtype=torch.float32, device=x.device)
    L = lib()
    ws = _ws.get(L.drl_agg_loss_workspace_bytes(B, R), x.device)
    check(L.drl_agg_loss(_p(x), _p(m), mask_dtype_code(m), B, R, _lib.AGG_MODES[loss_agg_mode], _p(out), _p(ws),
                         ws.numel(), _stream()), "drl_agg_loss")
    return out


# ----------------------------------------------------------------------------------------------- K2
def _logits_2d(logits):
    if logits.dtype not in _LOGIT_DTYPES:
        raise ValueError(f"logits dtype {logits.dtype} not supported (float32 / bfloat16)")
    if logits.dim() != 2:
        logits = logits.reshape(-1, logits.shape[-1])
    if logits.stride(-1) != 1:
        logits = logits.contiguous()
    return logits


def logprob_entropy_fwd(logits, labels, temperature=1.0, want_entropy=True, want_lse=True):
    _dev(logits, labels)
    lg = _logits_2d(logits)
    lab = _c(labels.reshape(-1).to(torch.int64))
    N, V = lg.shape
    dev = lg.device
    logp = torch.empty(N, dtype=torch.float32, device=dev)
    ent = torch.empty(N, dtype=torch.float32, device=dev) if want_entropy else None
    lse = torch.empty(N, dtype=torch.float32, device=dev) if want_lse else None
    check(lib().drl_logprob_entropy_fwd(_p(lg), _LOGIT_DTYPES[lg.dtype], N, V, lg.stride(0), _p(lab),
                                        float(temperature), _p(logp), _p(ent), _p(lse), _stream()),
          "drl_logprob_entropy_fwd")
    return logp, ent, lse


def logprob_entropy_bwd(logits, labels, temperature, dlogp, dentropy, lse, entropy, out=None, out_dtype=None):
    _dev(logits, labels)
    lg = _logits_2d(logits)
    lab = _c(labels.reshape(-1).to(torch.int64))
    N, V = lg.shape
    if out is None:
        out = torch.empty((N, V), dtype=out_dtype or lg.dtype, device=lg.device)
    dlogp = _c(dlogp.reshape(-1).float()) if dlogp is not None else None
    dentropy = _c(dentropy.reshape(-1).float()) if dentropy is not None else None
    check(lib().drl_logprob_entropy_bwd(_p(lg), _LOGIT_DTYPES[lg.dtype], N, V, lg.stride(0), _p(lab),
                                        float(temperature), _p(dlogp), _p(dentropy), _p(_c(lse)), _p(_c(entropy)),
                                        _p(out), _LOGIT_DTYPES[out.dtype], out.stride(0), _stream()),
          "drl_logprob_entropy_bwd")
    return out


# ----------------------------------------------------------------------------------------------- A21
def _pad_k64(t):
    """Zero-pad the hidden dimension to a multiple of 64 (the fused kernel's K step; zeros add nothing)."""
    H = t.shape[-1]
    return t if H % 64 == 0 else torch.nn.functional.pad(t, (0, 64 - H % 64))


def linear_logprob_fwd(hidden, weight, labels, temperature=1.0, want_entropy=True, want_lse=True):
    """Fused lm_head + log-prob + entropy (csrc/fused_linear.hip): hidden (N, H) bf16, weight (V, H) bf16,
    labels (N,) -> logp, entropy (or None), lse (or None), (N,) fp32; the (N, V) logits are never stored."""
    _dev(hidden, weight, labels)
    h, w = _pad_k64(hidden), _pad_k64(weight)
    assert h.dim() == 2 and h.stride(1) == 1 and w.is_contiguous() and h.dtype == w.dtype == torch.bfloat16
    lab = _c(labels.reshape(-1).to(torch.int64))
    N, H = h.shape
    V = w.shape[0]
    dev = h.device
    logp = torch.empty(N, dtype=torch.float32, device=dev)
    ent = torch.empty(N, dtype=torch.float32, device=dev) if want_entropy else None
    lse = torch.empty(N, dtype=torch.float32, device=dev) if want_lse else None
    nws = lib().drl_linear_logprob_workspace_bytes(N, H, V)
    ws = _ws.get(nws, dev)
    check(lib().drl_linear_logprob_fwd(_p(h), h.stride(0), _p(w), _p(lab), _lib.DRL_BF16, N, H, V, float(temperature),
                                       _p(logp), _p(ent), _p(lse), _p(ws), nws, _stream()), "drl_linear_logprob_fwd")
    return logp, ent, lse


def linear_logprob_dlogits(hidden, weight, labels, temperature, dlogp, dentropy, lse, entropy, out=None):
    """d_logits^T (V, N) bf16 of the fused lm_head log-prob / entropy (z recomputed on MFMA)."""
    _dev(hidden, weight, labels, dlogp, lse)
    h, w = _pad_k64(hidden), _pad_k64(weight)
    assert h.dim() == 2 and h.stride(1) == 1 and w.is_contiguous() and h.dtype == w.dtype == torch.bfloat16
    lab = _c(labels.reshape(-1).to(torch.int64))
    N, H = h.shape
    V = w.shape[0]
    if out is None:
        out = torch.empty(V, N, dtype=torch.bfloat16, device=h.device)
    assert out.shape == (V, N) and out.stride(1) == 1 and out.dtype == torch.bfloat16
    dlogp = _c(dlogp.reshape(-1).float())
    dentropy = _c(dentropy.reshape(-1).float()) if dentropy is not None else None
    check(lib().drl_linear_logprob_dlogits(_p(h), h.stride(0), _p(w), _p(lab), _lib.DRL_BF16, N, H, V, float(temperature),
                                           _p(dlogp), _p(dentropy), _p(_c(lse)), _p(_c(entropy)), _p(out),
                                           out.stride(0), _stream()), "drl_linear_logprob_dlogits")
    return out


# ----------------------------------------------------------------------------------------------- K3/K5
def grpo_outcome_advantage(token_level_rewards, response_mask, row_group, group_offsets, group_members, G,
                           epsilon=1e-6, norm_adv_by_std_in_grpo=True):
    _dev(token_level_rewards, response_mask, row_group, group_offsets, group_members)
    r, m = _c(token_level_rewards.float()), _c(response_mask)
    B, R = r.shape
    adv = torch.empty_like(r)
    ret = torch.empty_like(r)
    L = lib()
    ws = _ws.get(L.drl_grpo_workspace_bytes(B), r.device)
    check(L.drl_grpo_outcome_advantage(_p(r), _p(m), mask_dtype_code(m), _p(_c(row_group)), _p(_c(group_offsets)),
                                       _p(_c(group_members)), B, R, G, float(epsilon), int(bool(norm_adv_by_std_in_grpo)),
                                       _p(adv), _p(ret), _p(ws), ws.numel(), _stream()), "drl_grpo_outcome_advantage")
    return adv, ret


_GROUP_ESTIMATORS = {"grpo": 0, "rloo": 1, "reinforce_plus_plus_baseline": 2, "opo": 3, "gpg": 4, "grpo_passk": 5}


def group_outcome_advantage(estimator, token_level_rewards, response_mask, row_group, group_offsets, group_members, G,
                            epsilon=1e-6, norm_adv_by_std_in_grpo=True):
    """K3 over the uid-group CSR for GRPO / RLOO / REINFORCE++-baseline / OPO / GPG / GRPO pass@k
    (drl_group_outcome_advantage)."""
    _dev(token_level_rewards, response_mask, row_group, group_offsets, group_members)
    r, m = _c(token_level_rewards.float()), _c(response_mask)
    B, R = r.shape
    adv, ret = torch.empty_like(r), torch.empty_like(r)
    L = lib()
    ws = _ws.get(L.drl_group_outcome_advantage_workspace_bytes(B), r.device)
    check(L.drl_group_outcome_advantage(_p(r), _p(m), mask_dtype_code(m), _p(_c(row_group)), _p(_c(group_offsets)),
                                        _p(_c(group_members)), B, R, G, _GROUP_ESTIMATORS[estimator], float(epsilon),
                                        int(bool(norm_adv_by_std_in_grpo)), _p(adv), _p(ret), _p(ws), ws.numel(),
                                        _stream()), "drl_group_outcome_advantage")
    return adv, ret


def remax_advantage_return(token_level_rewards, reward_baselines, response_mask):
    """ReMax: reverse cumsum of masked rewards minus the greedy baseline (drl_remax_advantage_return)."""
    _dev(token_level_rewards, reward_baselines, response_mask)
    r, m = _c(token_level_rewards.float()), _c(response_mask)
    bl = _c(reward_baselines.float().reshape(-1))
    B, R = r.shape
    assert bl.numel() == B
    adv, ret = torch.empty_like(r), torch.empty_like(r)
    check(lib().drl_remax_advantage_return(_p(r), _p(bl), _p(m), mask_dtype_code(m), B, R, _p(adv), _p(ret), _stream()),
          "drl_remax_advantage_return")
    return adv, ret


def reinforce_pp_advantage_return(token_level_rewards, response_mask, gamma):
    _dev(token_level_rewards, response_mask)
    r, m = _c(token_level_rewards.float()), _c(response_mask)
    B, R = r.shape
    adv, ret = torch.empty_like(r), torch.empty_like(r)
    L = lib()
    ws = _ws.get(L.drl_gae_workspace_bytes(B, R), r.device)
    check(L.drl_reinforce_pp_advantage_return(_p(r), _p(m), mask_dtype_code(m), B, R, float(gamma), _p(adv), _p(ret),
                                              _p(ws), ws.numel(), _stream()), "drl_reinforce_pp_advantage_return")
    return adv, ret


def gae_advantage_return(token_level_rewards, values, response_mask, gamma, lam):
    _dev(token_level_rewards, values, response_mask)
    r, m = _c(token_level_rewards.float()), _c(response_mask)
    v = _c(values if values.dtype == torch.bfloat16 else values.float())  # bf16 critic values read as stored
    B, R = r.shape
    adv, ret = torch.empty_like(r), torch.empty_like(r)
    L = lib()
    ws = _ws.get(L.drl_gae_workspace_bytes(B, R), r.device)
    check(L.drl_gae_advantage_return(_p(r), _p(v), _VALUE_DTYPES[v.dtype], _p(m), mask_dtype_code(m), B, R, float(gamma),
                                     float(lam), _p(adv), _p(ret), _p(ws), ws.numel(), _stream()),
          "drl_gae_advantage_return")
    return adv, ret


# ----------------------------------------------------------------------------------------------- K6 critic
_VALUE_DTYPES = {torch.float32: _lib.DRL_F32, torch.bfloat16: _lib.DRL_BF16}


def value_loss_fwd_bwd(vpreds, values, returns, response_mask, *, cliprange_value, loss_agg_mode="token-mean",
                       loss_scale_factor=1.0, want_dvpreds=True, out=None):
    """One launch after a row-count pre-pass: float32[8] scalars (DRL_VALUE_OUT_*: vf_loss, vf_clipfrac,
    vpred_mean, loss = vf_loss * loss_scale_factor, mask count) and d loss / d vpreds (float32)."""
    _dev(vpreds, values, returns, response_mask)
    if vpreds.dtype != values.dtype:
        values = values.to(vpreds.dtype)
    if vpreds.dtype not in _VALUE_DTYPES:
        raise TypeError(f"vpreds dtype {vpreds.dtype}: float32 or bfloat16")
    vp, vo, rt, m = _c(vpreds.detach()), _c(values), _c(returns.float()), _c(response_mask)
    B, R = vp.shape
    assert vo.shape == (B, R) and rt.shape == (B, R) and m.shape == (B, R)
    prm = _lib.ValueLossParams(float(cliprange_value), float(loss_scale_factor), _lib.AGG_MODES[loss_agg_mode], 0)
    dev = vp.device
    if out is None:
        out = torch.empty(_lib.VALUE_OUT_N, dtype=torch.float32, device=dev)
    dv = torch.empty(B, R, dtype=torch.float32, device=dev) if want_dvpreds else None
    L = lib()
    ws = _ws.get(L.drl_value_loss_workspace_bytes(B, R), dev)
    check(L.drl_value_loss_fwd_bwd(_p(vp), _p(vo), _VALUE_DTYPES[vp.dtype], _p(rt), _p(m), mask_dtype_code(m), B, R,
                                   ctypes.byref(prm), _p(out), _p(dv), _p(ws), ws.numel(), _stream()),
          "drl_value_loss_fwd_bwd")
    return out, dv


def value_head_fwd(hidden, weight, bias, out_dtype=None):
    """values (N,) = hidden (N, H) . weight (H) + bias, fp32 accumulation, stored as ``out_dtype``
    (default: the hidden dtype, as the reference's autocast Linear)."""
    _dev(hidden, weight, bias)
    assert hidden.dim() == 2 and hidden.stride(-1) == 1
    N, H = hidden.shape
    dt = _VALUE_DTYPES[hidden.dtype]
    w = _c(weight.reshape(-1).to(hidden.dtype))
    b = _c(bias.reshape(-1).to(hidden.dtype)) if bias is not None else None
    od = out_dtype or hidden.dtype
    out = torch.empty(N, dtype=od, device=hidden.device)
    check(lib().drl_value_head_fwd(_p(hidden), hidden.stride(0), _p(w), _p(b), dt, N, H, _p(out), _VALUE_DTYPES[od],
                                   _stream()), "drl_value_head_fwd")
    return out


def value_head_bwd(hidden, weight, dvalues, dweight=None, dbias=None, want_dhidden=True):
    """dhidden (N, H) in the hidden dtype; accumulates into the fp32 ``dweight`` (H) / ``dbias`` (1)."""
    _dev(hidden, weight, dvalues, dweight, dbias)
    N, H = hidden.shape
    dt = _VALUE_DTYPES[hidden.dtype]
    w = _c(weight.reshape(-1).to(hidden.dtype))
    dv = _c(dvalues.reshape(-1).float())
    for g in (dweight, dbias):
        assert g is None or (g.dtype == torch.float32 and g.is_contiguous())
    dh = torch.empty(N, H, dtype=hidden.dtype, device=hidden.device) if want_dhidden else None
    L = lib()
    ws = _ws.get(L.drl_value_head_bwd_workspace_bytes(N, H), hidden.device)
    check(L.drl_value_head_bwd(_p(hidden), hidden.stride(0), _p(w), dt, _p(dv), N, H, _p(dh), H if dh is not None else 0,
                               _p(dweight), _p(dbias), _p(ws), ws.numel(), _stream()), "drl_value_head_bwd")
    return dh


# ----------------------------------------------------------------------------------------------- K4
def select_tokens(logits, out_tokens, *, do_sample=False, temperature=1.0, top_k=0, top_p=1.0, seed=0, step=0,
                  row_base=0, pad_token_id=0, eos_ids=None, unfinished=None, dev_step=None):
    """Pick one token per row into ``out_tokens`` (int64 view with any row stride, e.g. responses[:, t]).

    ``dev_step`` (device int64 scalar s): the Philox offset becomes step + s and row n's token goes to
    ``out_tokens[n * stride + s]`` — the graph-captured decode loop passes ``responses[:, 0]`` and s."""
    _dev(logits, out_tokens, eos_ids, unfinished)
    lg = _logits_2d(logits)
    N, V = lg.shape
    assert out_tokens.dtype == torch.int64 and out_tokens.numel() == N
    ld_out = out_tokens.stride(0) if out_tokens.dim() == 1 else 1
    # N u64 greedy maxima + N f32 top-k / top-p cuts + (N, ceil(V / 2048)) sampling slice masses
    ws = _select_workspace(lg.device, (lib().drl_select_tokens_workspace_bytes(N, V) + 7) // 8)
    prm = _lib.SamplingParams(int(bool(do_sample)), float(temperature), int(top_k), float(top_p),
                              int(seed) & 0xFFFFFFFFFFFFFFFF, int(step), int(row_base), int(pad_token_id),
                              None if eos_ids is None else eos_ids.data_ptr(),
                              0 if eos_ids is None else eos_ids.numel(),
                              None if dev_step is None else dev_step.data_ptr())
    check(lib().drl_select_tokens(_p(lg), _LOGIT_DTYPES[lg.dtype], N, V, lg.stride(0), ctypes.byref(prm),
                                  _p(unfinished), _p(out_tokens), ld_out, _p(ws), ws.numel() * 8, _stream()),
          "drl_select_tokens")
    return out_tokens


def linear_select_tokens(hidden, weight, out_tokens, *, do_sample=False, temperature=1.0, top_k=0, top_p=1.0, seed=0,
                         step=0, row_base=0, pad_token_id=0, eos_ids=None, unfinished=None, dev_step=None):
    """select_tokens on the bf16 logits hidden @ weight^T without writing them (lm_head fused with K4,
    csrc/fused_linear.hip): hidden (N, H) bf16, weight (V, H) bf16, H % 64 == 0."""
    _dev(hidden, weight, out_tokens, eos_ids, unfinished)
    assert hidden.dim() == 2 and hidden.stride(1) == 1 and weight.is_contiguous()
    assert hidden.dtype == weight.dtype == torch.bfloat16
    N, H = hidden.shape
    V = weight.shape[0]
    assert out_tokens.dtype == torch.int64 and out_tokens.numel() == N
    ld_out = out_tokens.stride(0) if out_tokens.dim() == 1 else 1
    ws = _select_workspace(hidden.device, N)
    prm = _lib.SamplingParams(int(bool(do_sample)), float(temperature), int(top_k), float(top_p),
                              int(seed) & 0xFFFFFFFFFFFFFFFF, int(step), int(row_base), int(pad_token_id),
                              None if eos_ids is None else eos_ids.data_ptr(),
                              0 if eos_ids is None else eos_ids.numel(),
                              None if dev_step is None else dev_step.data_ptr())
    check(lib().drl_linear_select_tokens(_p(hidden), hidden.stride(0), _p(weight), _lib.DRL_BF16, N, H, V,
                                         ctypes.byref(prm), _p(unfinished), _p(out_tokens), ld_out, _p(ws),
                                         ws.numel() * 8, _stream()), "drl_linear_select_tokens")
    return out_tokens


def token_logprob(logits, tokens, out, temperature=1.0, dev_step=None):
    """rollout.calculate_log_probs: out[n, s] = log softmax(logits[n] / T)[tokens[n, s]] for the column s =
    ``dev_step`` (device int64 scalar; 0 when None) of the (N, *) int64 ``tokens`` / fp32 ``out`` views."""
    _dev(logits, tokens, out, dev_step)
    lg = _logits_2d(logits)
    N, V = lg.shape
    assert tokens.dtype == torch.int64 and out.dtype == torch.float32
    assert tokens.shape[0] == N and out.shape[0] == N
    ld_tok = tokens.stride(0) if tokens.dim() > 1 or tokens.numel() > 1 else 1
    ld_out = out.stride(0) if out.dim() > 1 or out.numel() > 1 else 1
    check(lib().drl_token_logprob(_p(lg), _LOGIT_DTYPES[lg.dtype], N, V, lg.stride(0), _p(tokens), ld_tok,
                                  _p(dev_step), float(temperature), _p(out), ld_out, _stream()), "drl_token_logprob")
    return out


_SELECT_WS = {}


def _select_workspace(device, N):
    """Per-device zeroed int64 buffer (>= N rows) that the selection kernels leave zeroed after each call
    (valid inside captured graphs: calls on one stream reuse it in order)."""
    key = (str(device), _lane())
    ws = _SELECT_WS.get(key)
    if ws is None or ws.numel() < N:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("select_tokens: call once outside graph capture to size its workspace")
        ws = torch.zeros(max(N, 1024), dtype=torch.int64, device=device)
        _SELECT_WS[key] = ws
    return ws


def response_mask(responses, eos_ids, dtype=torch.int64, out=None):
    _dev(responses, eos_ids)
    B, R = responses.shape
    if out is None:
        out = torch.empty((B, R), dtype=dtype, device=responses.device)
    code = {torch.int64: _lib.DRL_I64, torch.int32: _lib.DRL_I32, torch.uint8: _lib.DRL_U8, torch.bool: _lib.DRL_U8,
            torch.float32: _lib.DRL_F32}[out.dtype]
    check(lib().drl_response_mask(_p(responses), B, R, responses.stride(0), _p(eos_ids), eos_ids.numel(), _p(out),
                                  code, out.stride(0), _stream()), "drl_response_mask")
    return out


def position_ids(attention_mask):
    _dev(attention_mask)
    m = _c(attention_mask)
    B, T = m.shape
    out = torch.empty((B, T), dtype=torch.int64, device=m.device)
    check(lib().drl_position_ids(_p(m), mask_dtype_code(m), B, T, _p(out), _stream()), "drl_position_ids")
    return out


def response_position_ids_(position_ids_full, prompt_len):
    """In place: fill columns [prompt_len:] of a (B, P+R) int64 buffer from column prompt_len-1."""
    _dev(position_ids_full)
    assert position_ids_full.is_contiguous() and position_ids_full.dtype == torch.int64
    B, T = position_ids_full.shape
    check(lib().drl_response_position_ids(_p(position_ids_full), B, prompt_len, T - prompt_len, _stream()),
          "drl_response_position_ids")
    return position_ids_full


# ----------------------------------------------------------------------------------------------- A15
def grad_norm(flat_grads, out=None):
    _dev(flat_grads)
    assert flat_grads.is_contiguous() and flat_grads.dtype == torch.float32
    if out is None:
        out = torch.empty(1, dtype=torch.float32, device=flat_grads.device)
    L = lib()
    ws = _ws.get(L.drl_grad_norm_workspace_bytes(flat_grads.numel()), flat_grads.device)
    check(L.drl_grad_norm(_p(flat_grads), flat_grads.numel(), _p(out), _p(ws), ws.numel(), _stream()), "drl_grad_norm")
    return out


def adamw_step(params, grads, exp_avg, exp_avg_sq, *, lr, beta1, beta2, eps, weight_decay, step, max_grad_norm,
               grad_norm_t=None, params_bf16=None):
    _dev(params, grads, exp_avg, exp_avg_sq, grad_norm_t, params_bf16)
    hp = _lib.AdamWParams(float(lr), float(beta1), float(beta2), float(eps), float(weight_decay), int(step),
                          float(max_grad_norm))
    check(lib().drl_adamw_step(_p(params), _p(grads), _p(exp_avg), _p(exp_avg_sq), _p(params_bf16), params.numel(),
                               ctypes.byref(hp), _p(grad_norm_t), _stream()), "drl_adamw_step")


# ----------------------------------------------------------------------------------------------- layers
def _edt(t):
    try:
        return _LOGIT_DTYPES[t.dtype]
    except KeyError as e:
        raise ValueError(f"activation dtype {t.dtype} not supported (bfloat16 / float32)") from e


def rope_qkv_fwd(qkv, position_ids, cos_t, sin_t, Hq, Hkv, D, q, k, v, koff=0, koff_dev=None, vt=None, qt=None,
                 kt=None, src_rows=None, q_skip=None):
    """qkv (B,T,(Hq+2Hkv)D) -> q (B,Hkv,G,T,D); k, v written at [:, :, koff:koff+T] of (B,Hkv,Tk,D).

    ``koff_dev`` (device int64 scalar) replaces ``koff`` for graph-captured decode steps. ``qt`` (B,Hkv,G,D,ld),
    ``kt`` / ``vt`` (B,Hkv,D,ld): head-dim-major copies for the fused attention kernels (same ld). ``src_rows``
    (B*T,) int64: qkv is packed (nnz, (Hq+2Hkv)D) and position (b, t) reads row src_rows[b*T+t] (< 0: zeros) —
    drl_rope_qkv_fwd_rows, no padded copy of qkv; B, T then come from ``position_ids``. ``q_skip`` (B,) int32: the
    ``q_start`` of the fused attention that reads q — rows t < q_skip[b] & ~31 are left unwritten (never read)."""
    if src_rows is not None:
        B, T = position_ids.shape[0], position_ids.shape[1]
        assert qkv.dim() == 2 and qkv.is_contiguous() and src_rows.dtype == torch.int64 and src_rows.numel() == B * T
        _dev(src_rows)
    else:
        B, T = qkv.shape[0], qkv.shape[1]
    lds = {(vt_ld(t) if t is vt else t.stride(-2)) for t in (qt, kt, vt) if t is not None}
    if vt is not None:
        _vt_cap_ok(vt, k.shape[2])
    assert len(lds) <= 1, "qt / kt / vt must share their row stride"
    if q_skip is not None:
        assert q_skip.dtype == torch.int32 and q_skip.numel() == B and q_skip.is_contiguous()
        _dev(q_skip)
    check(lib().drl_rope_qkv_fwd_rows(_p(qkv), _p(src_rows), _edt(qkv), _p(position_ids), _p(cos_t), _p(sin_t),
                                      cos_t.shape[0], B, T, Hq, Hkv, D, _p(q), _p(k), _p(v), k.shape[2], koff,
                                      _p(koff_dev), _p(qt), _p(kt), _p(vt), lds.pop() if lds else 0, _p(q_skip),
                                      _stream()),
          "drl_rope_qkv_fwd")


def rope_qkv_bwd(dq, dk, dv, position_ids, cos_t, sin_t, Hq, Hkv, D, dqkv):
    B, T = dqkv.shape[0], dqkv.shape[1]
    check(lib().drl_rope_qkv_bwd(_p(dq), _p(dk), _p(dv), _edt(dq), _p(position_ids), _p(cos_t), _p(sin_t),
                                 cos_t.shape[0], B, T, Hq, Hkv, D, _p(dqkv), _stream()), "drl_rope_qkv_bwd")


def masked_softmax_fwd(scores_f32, probs, key_valid_u8, B, HG, Tq, Tk, qoff, scale):
    """fp32 scores (B,Hkv,G,Tq,Tk) -> probs (activation dtype)."""
    assert scores_f32.dtype == torch.float32
    check(lib().drl_masked_softmax_fwd(_p(scores_f32), _p(probs), _edt(probs), _p(key_valid_u8),
                                       key_valid_u8.stride(0), B, HG, Tq, Tk, qoff, float(scale), _stream()),
          "drl_masked_softmax_fwd")


def masked_softmax_bwd(probs, dprobs_f32, dscores, rows, Tk, scale):
    assert dprobs_f32.dtype == torch.float32
    check(lib().drl_masked_softmax_bwd(_p(probs), _p(dprobs_f32), _p(dscores), _edt(probs), rows, Tk, float(scale),
                                       _stream()), "drl_masked_softmax_bwd")


def add_rmsnorm_fwd(x_in, delta, x_out, weight, y, rstd, eps):
    N, H = x_in.numel() // x_in.shape[-1], x_in.shape[-1]
    check(lib().drl_add_rmsnorm_fwd(_p(x_in), _p(delta), _p(x_out), _p(weight), _p(y), _edt(y), _p(rstd), N, H,
                                    float(eps), _stream()), "drl_add_rmsnorm_fwd")


def rmsnorm_bwd(x, weight, rstd, dy, dx, dw, dx_in="inplace", dx_bf16=None):
    """dx = dx_in + RMSNorm backward of dy (dx_in "inplace": dx itself, None: zero); dw += its weight gradient;
    dx_bf16 (optional) receives bf16(dx) from the same pass."""
    N, H = x.numel() // x.shape[-1], x.shape[-1]
    L = lib()
    ws = _ws.get(L.drl_rmsnorm_bwd_workspace_bytes(N, H), x.device)
    src = dx if isinstance(dx_in, str) else dx_in
    for t in (src, dx_bf16):
        assert t is None or (t.is_contiguous() and t.numel() == dx.numel())
    assert dx_bf16 is None or dx_bf16.dtype == torch.bfloat16
    check(L.drl_rmsnorm_bwd_ex(_p(x), _p(weight), _p(rstd), _p(dy), _edt(dy), _p(src), _p(dx), _p(dx_bf16), _p(dw), N,
                               H, _p(ws), ws.numel(), _stream()), "drl_rmsnorm_bwd_ex")


def swiglu_fwd(gate_up, out):
    N, I2 = gate_up.numel() // gate_up.shape[-1], gate_up.shape[-1]
    check(lib().drl_swiglu_fwd(_p(gate_up), _p(out), _edt(gate_up), N, I2 // 2, _stream()), "drl_swiglu_fwd")


def swiglu_bwd(gate_up, dout, dgate_up):
    N, I2 = gate_up.numel() // gate_up.shape[-1], gate_up.shape[-1]
    check(lib().drl_swiglu_bwd(_p(gate_up), _p(dout), _p(dgate_up), _edt(gate_up), N, I2 // 2, _stream()),
          "drl_swiglu_bwd")


def decode_attention(q, k_cache, v_cache, key_valid, L, out, qpos=None, qpos_dev=None, split=True):
    """q (B,Hkv,G,D) one token; caches (B,Hkv,Tk,D); keys j < L with key_valid[b,j] and j <= qpos -> out."""
    _dev(q, k_cache, v_cache, key_valid, out)
    B, Hkv, G, D = q.shape
    Tk = k_cache.shape[2]
    assert k_cache.is_contiguous() and v_cache.is_contiguous() and q.is_contiguous() and out.is_contiguous()
    assert key_valid.dtype == torch.uint8 and key_valid.stride(1) == 1 and key_valid.shape[0] == B
    qp = L - 1 if qpos is None else int(qpos)
    Lb = lib()
    nb = Lb.drl_decode_attention_workspace_bytes(B, Hkv, G, D, L) if split else 0
    ws = _ws.get(nb, q.device) if nb else None
    check(Lb.drl_decode_attention(_p(q), _p(k_cache), _p(v_cache), _edt(q), _p(key_valid), key_valid.stride(0),
                                  _p(qpos_dev), qp, B, Hkv, G, D, Tk, L, 1.0 / math.sqrt(D), _p(out), _p(ws), nb,
                                  _stream()), "drl_decode_attention")
    return out


DRL_VT_BLOCKED = -32  # include/dotsrl_amd.h: ld_vt of the key-blocked V^T cache layout


def vt_ld(vt):
    """ld_vt of a V^T operand: its row stride (B, Hkv, D, ld), or DRL_VT_BLOCKED for the key-blocked cache layout
    (B, Hkv, ceil(cap / 32), D, 32) that KVCache keeps (one 32-key block's V^T contiguous)."""
    if vt.dim() == 5:
        assert vt.shape[-1] == 32 and vt.is_contiguous(), "key-blocked V^T must be a contiguous (B, Hkv, NB, D, 32)"
        return DRL_VT_BLOCKED
    assert vt.stride(-1) == 1 and vt.stride(-2) * vt.shape[-2] == vt.stride(-3)
    return vt.stride(-2)


def vt_blocked_to_plain(vt):
    """(B, Hkv, NB, D, 32) key-blocked V^T -> (B, Hkv, D, NB * 32) head-dim-major copy (tests / inspection)."""
    B, Hkv, NB, D, _ = vt.shape
    return vt.permute(0, 1, 3, 2, 4).reshape(B, Hkv, D, NB * 32)


def _vt_cap_ok(vt, cap):
    assert vt.dim() != 5 or vt.shape[2] == (cap + 31) // 32, "key-blocked V^T must hold ceil(K capacity / 32) blocks"


def flash_attn_fwd(q, k, vt, key_valid, out, Tk=None, qoff=0, lse=None, q_start=None, out_rows=None):
    """Fused causal + key-padding attention (MFMA). q (B,Hkv,G,Tq,D) bf16, k (B,Hkv,>=Tk,D) (keys [0,Tk) used),
    vt (B,Hkv,D,ld) with ld >= Tk a multiple of 8; out (B,Tq,Hkv*G*D); lse optional (B,Hkv,G,Tq) fp32;
    q_start optional (B,) int32: query tiles of row b wholly below q_start[b] skipped (rows left unwritten).
    ``out_rows`` (B*Tq,) int64: out is packed (rows, Hkv*G*D) and query (b, t) writes row out_rows[b*Tq+t] (< 0: not
    written) — drl_flash_attn_fwd_rows."""
    _dev(q, k, vt, key_valid, out, lse, q_start, out_rows)
    assert q_start is None or (q_start.dtype == torch.int32 and q_start.numel() == q.shape[0])
    B, Hkv, G, Tq, D = q.shape
    Tk = k.shape[2] if Tk is None else Tk
    assert q.is_contiguous() and k.is_contiguous() and out.is_contiguous()
    assert key_valid.dtype == torch.uint8 and key_valid.stride(1) == 1
    if out_rows is not None:
        assert out_rows.dtype == torch.int64 and out_rows.numel() == B * Tq and out_rows.is_contiguous()
        assert out.dim() == 2 and out.shape[1] == Hkv * G * D
    _vt_cap_ok(vt, k.shape[2])
    check(lib().drl_flash_attn_fwd_rows(_p(q), _p(k), _p(vt), _edt(q), _p(key_valid), key_valid.stride(0), B, Hkv, G,
                                        D, Tq, Tk, k.shape[2], vt_ld(vt), qoff, _p(q_start), 1.0 / math.sqrt(D),
                                        _p(out), _p(out_rows), _p(lse), _stream()),
          "drl_flash_attn_fwd")
    return out


def flash_attn_bwd(q, k, kt, v, o, dout, lse, key_valid, dq, dk, dv, q_start=None, o_rows=None):
    """Backward of flash_attn_fwd (Tq == Tk, qoff 0): q (B,Hkv,G,T,D), k/v (B,Hkv,T,D), kt (B,Hkv,D,ld),
    o/dout (B,T,Hq*D), lse (B,Hkv,G,T) -> dq (B,Hkv,G,T,D), dk/dv (B,Hkv,T,D). q_start as in the forward (dout
    zero on the skipped tiles). ``o_rows`` (B*T,) int64: o is the packed (rows, Hq*D) output the forward wrote
    through the same map (drl_flash_attn_bwd_rows; dout zero at the map's negative entries)."""
    _dev(q, k, kt, v, o, dout, lse, key_valid, dq, dk, dv, q_start, o_rows)
    if o_rows is not None:
        assert o_rows.dtype == torch.int64 and o_rows.numel() == q.shape[0] * q.shape[3] and o_rows.is_contiguous()
    assert q_start is None or (q_start.dtype == torch.int32 and q_start.numel() == q.shape[0])
    B, Hkv, G, T, D = q.shape
    assert kt.stride(-1) == 1 and kt.stride(-2) * D == kt.stride(1)
    for t in (q, k, v, o, dout, lse, dq, dk, dv):
        assert t.is_contiguous()
    delta = _ws.get(B * Hkv * G * T * 4, q.device)
    check(lib().drl_flash_attn_bwd_rows(_p(q), _p(k), _p(kt), _p(v), _p(o), _p(o_rows), _p(dout), _p(lse), _edt(q),
                                        _p(key_valid), key_valid.stride(0), B, Hkv, G, D, T, kt.stride(-2),
                                        _p(q_start), 1.0 / math.sqrt(D), _p(delta), _p(dq), _p(dk), _p(dv), _stream()),
          "drl_flash_attn_bwd")


def colsum_bf16_acc(x, out):
    """out (C,) fp32 += x (N, C) bf16 summed over rows (csrc/layers.hip, deterministic)."""
    _dev(x, out)
    assert x.dim() == 2 and x.stride(1) == 1 and x.dtype == torch.bfloat16 and out.dtype == torch.float32
    N, C = x.shape
    assert out.numel() == C and out.is_contiguous()
    L = lib()
    ws = _ws.get(L.drl_colsum_bf16_workspace_bytes(N, C), x.device)
    check(L.drl_colsum_bf16_acc(_p(x), x.stride(0), N, C, _p(out), _p(ws), ws.numel(), _stream()), "drl_colsum_bf16_acc")
    return out


GEMM_PLAIN, GEMM_BIAS, GEMM_SWIGLU, GEMM_SWIGLU_BWD = 0, 1, 2, 3


def copy_rows(src, dst, src_idx=None, dst_idx=None, n=None):
    """dst[dst_idx[i]] = src[src_idx[i]] row by row (identity where an index is None; a negative index skips the row)
    — the remove-padding gathers / scatters (csrc/rows.hip)."""
    _dev(src, dst, src_idx, dst_idx)
    assert src.dim() == 2 and dst.dim() == 2 and src.stride(1) == 1 and dst.stride(1) == 1
    assert src.dtype == dst.dtype and src.shape[1] == dst.shape[1]
    if n is None:
        n = (src_idx if src_idx is not None else dst_idx if dst_idx is not None else src).shape[0]
    for ix in (src_idx, dst_idx):
        assert ix is None or (ix.dtype == torch.int64 and ix.is_contiguous() and ix.numel() >= n)
    es = src.element_size()
    check(lib().drl_copy_rows(_p(src), src.stride(0) * es, _p(src_idx), _p(dst), dst.stride(0) * es, _p(dst_idx), n,
                              src.shape[1] * es, _stream()), "drl_copy_rows")
    return dst


def gather_rows_zero(src, dst, src_idx):
    """dst[i] = src[src_idx[i]] for every row i of dst, a zero row where src_idx[i] < 0 (csrc/rows.hip,
    drl_gather_rows): pad_input's zero pad rows written by the gather itself, so ``dst`` may be uninitialised."""
    _dev(src, dst, src_idx)
    assert src.dim() == 2 and dst.dim() == 2 and src.stride(1) == 1 and dst.stride(1) == 1
    assert src.dtype == dst.dtype and src.shape[1] == dst.shape[1]
    n = dst.shape[0]
    assert src_idx.dtype == torch.int64 and src_idx.is_contiguous() and src_idx.numel() >= n
    es = src.element_size()
    check(lib().drl_gather_rows(_p(src), src.stride(0) * es, _p(src_idx), _p(dst), dst.stride(0) * es, n,
                                src.shape[1] * es, _stream()), "drl_gather_rows")
    return dst


def sum_rows(src, src_idx, dst, dst_idx=None):
    """dst[dst_idx[j]] = sum_k src[src_idx[k, j]] for src_idx (K, m) (entries < 0 add nothing), fp32 accumulation in
    k order (csrc/rows.hip): the gradient of a packed row read by several padded positions (prefix sharing)."""
    _dev(src, dst, src_idx, dst_idx)
    assert src.dim() == 2 and dst.dim() == 2 and src.stride(1) == 1 and dst.stride(1) == 1
    assert src.dtype == dst.dtype and src.shape[1] == dst.shape[1] and src_idx.dim() == 2
    K, m = src_idx.shape
    for ix in (src_idx, dst_idx):
        assert ix is None or (ix.dtype == torch.int64 and ix.is_contiguous())
    assert dst_idx is None or dst_idx.numel() == m
    check(lib().drl_sum_rows(_p(src), src.stride(0), _p(src_idx), K, _p(dst), dst.stride(0), _p(dst_idx), m,
                             src.shape[1], _edt(src), _stream()), "drl_sum_rows")
    return dst


LAYOUT_K, LAYOUT_T = 0, 1


class _GemmWorkspace:
    """drl_gemm's stream-K slabs + flag words, one per (device, slot), zeroed once at allocation (every call leaves
    the flag words zero again); calls of one slot share it in stream order. Slot 1 belongs to the side stream of
    qwen2.dgrad_wgrad (a weight gradient running concurrently with its input gradient)."""

    def __init__(self):
        self.buf = {}

    def get(self, device, slot=0):
        if slot == 0 and _lane():
            slot = ("lane", _lane())
        key = (device.index if device.index is not None else torch.cuda.current_device(), slot)
        b = self.buf.get(key)
        if b is None:
            n = lib().drl_gemm_workspace_bytes()
            if n <= 0:
                raise RuntimeError(f"drl_gemm_workspace_bytes: {n}")
            b = torch.zeros(n, dtype=torch.uint8, device=device)
            self.buf[key] = b
        return b


_ws_gemm = _GemmWorkspace()


def gemm(a, a_layout, b, b_layout, M, N, K, out, beta=False, bias=None, swiglu=False, out_gu=None, ws_slot=0):
    """drl_gemm (csrc/gemm_sk.hip): out (M, N) (+)= sum_k A(m, k) B(n, k) with A(m, k) = a[m, k] (LAYOUT_K) or
    a[k, m] (LAYOUT_T), B likewise; bf16 operands, fp32 accumulation; ``out`` bf16 (+ bias / SwiGLU epilogues) or
    fp32 (``beta``: accumulate into it)."""
    _dev(a, b, out, bias, out_gu)
    assert a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and a.dim() == 2 and b.dim() == 2
    assert a.stride(1) == 1 and b.stride(1) == 1 and out.stride(1) == 1
    assert (a.shape == (M, K) if a_layout == LAYOUT_K else a.shape == (K, M)), (a.shape, M, K)
    assert (b.shape == (N, K) if b_layout == LAYOUT_K else b.shape == (K, N)), (b.shape, N, K)
    c_dt = _lib.DRL_F32 if out.dtype == torch.float32 else _lib.DRL_BF16
    assert out.dtype in (torch.float32, torch.bfloat16)
    assert out.shape == (M, N // 2 if swiglu else N), (out.shape, M, N)
    if out_gu is not None:
        assert swiglu and out_gu.shape == (M, N) and out_gu.stride(1) == 1
    if bias is not None:
        assert bias.is_contiguous() and bias.numel() == N
    epi = GEMM_SWIGLU if swiglu else (GEMM_BIAS if bias is not None else GEMM_PLAIN)
    ws = _ws_gemm.get(out.device, ws_slot)
    check(lib().drl_gemm(_p(a), a.stride(0), a_layout, _p(b), b.stride(0), b_layout, _p(out), out.stride(0), c_dt,
                         1 if beta else 0, M, N, K, _p(bias), epi, _p(out_gu),
                         out_gu.stride(0) if out_gu is not None else 0, _p(ws), ws.numel(), _stream()), "drl_gemm")
    return out


@functools.lru_cache(maxsize=4096)
def gemm_plan(M, N, K, epilogue=0, cus=256):
    """drl_gemm's decomposition of one launch (host-only arithmetic, csrc/gemm_sk.hip plan_decomposition):
    (mode, splits, grid, dp_tiles, sk_base) — mode 1 stream-K, 2 whole tiles (splits > 1: tail split-K), 3 split-K."""
    info = (ctypes.c_int32 * 5)()
    check(lib().drl_gemm_plan(M, N, K, epilogue, cus, info), "drl_gemm_plan")
    return tuple(info)


def gemm_spins(M, N, K, epilogue=0, cus=256):
    """True when the launch's plan has workgroups that spin-wait on other workgroups (stream-K, split-K, or whole tiles
    with a split-K tail): such a launch must not run beside another spinning drl_gemm launch (csrc/gemm_sk.hip header,
    co-residency rule (c))."""
    mode, splits = gemm_plan(M, N, K, epilogue, cus)[:2]
    return mode in (1, 3) or splits > 1


def gemm_timeout_word(device=None, slot=0):
    """The residency-timeout word of a drl_gemm workspace slot (0 unless a spin-wait gave up)."""
    device = torch.device("cuda", torch.cuda.current_device()) if device is None else device
    ws = _ws_gemm.get(device, slot)
    n = lib().drl_gemm_workspace_bytes()
    cus = (n - 256) // (256 * 256 * 4 + 4)
    return int(ws[cus * 256 * 256 * 4:].view(torch.int32)[cus])


def _pad_to_64(t, dim):
    """drl_gemm reduces K in steps of 64 (unless both operands are layout T): a 2-D operand whose reduction extent
    (``dim``) is not a multiple of 64 gets a zero-padded device copy — zero products leave every fp32 sum exact.
    Only models with such widths take it (every config of BASELINE.json has H, I, Hq*D multiples of 64)."""
    n = t.shape[dim]
    if n % 64 == 0:
        return t
    pad = (0, 64 - n % 64) if dim == 1 else (0, 0, 0, 64 - n % 64)
    return torch.nn.functional.pad(t, pad)


def linear_fwd(x, w, bias=None, swiglu=False, out=None, out_gu=None):
    """y = x W^T (+ bias) / SwiGLU(x [Wg | Wu]^T): x (M, K), w (N, K) -> (M, N) or (M, N / 2) bf16."""
    x, w = _pad_to_64(x, 1), _pad_to_64(w, 1)
    M, K = x.shape
    N = w.shape[0]
    if out is None:
        out = torch.empty(M, N // 2 if swiglu else N, dtype=torch.bfloat16, device=x.device)
    return gemm(x, LAYOUT_K, w, LAYOUT_K, M, N, K, out, bias=bias, swiglu=swiglu, out_gu=out_gu)


def linear_dgrad(dy, w, out=None):
    """dx = dy W (F.linear's grad_input): dy (M, N_out) bf16, w (N_out, N_in) read in place -> (M, N_in) bf16."""
    dy, w = _pad_to_64(dy, 1), _pad_to_64(w, 0)
    M, K = dy.shape
    N = w.shape[1]
    if out is None:
        out = torch.empty(M, N, dtype=torch.bfloat16, device=dy.device)
    return gemm(dy, LAYOUT_K, w, LAYOUT_T, M, N, K, out)


def linear_dgrad_swiglu_bwd(dy, w, gu, out=None):
    """The down_proj input gradient fused with the SwiGLU backward: da = bf16(dy W) (dy (M, H), w (H, I) read in
    place) -> dgu (M, 2I) = swiglu_bwd(gu, da) with gu (M, 2I) = the forward's [gate | up] (csrc/gemm_sk.hip)."""
    _dev(dy, w, gu)
    dy, w = _pad_to_64(dy, 1), _pad_to_64(w, 0)
    M, K = dy.shape
    N = w.shape[1]
    assert dy.dtype == w.dtype == gu.dtype == torch.bfloat16 and dy.stride(1) == 1 and w.stride(1) == 1
    assert gu.shape == (M, 2 * N) and gu.stride(1) == 1 and w.shape[0] == K
    if out is None:
        out = torch.empty(M, 2 * N, dtype=torch.bfloat16, device=dy.device)
    assert out.shape == (M, 2 * N) and out.stride(1) == 1
    ws = _ws_gemm.get(out.device)
    check(lib().drl_gemm(_p(dy), dy.stride(0), LAYOUT_K, _p(w), w.stride(0), LAYOUT_T, _p(out), out.stride(0),
                         _lib.DRL_BF16, 0, M, N, K, None, GEMM_SWIGLU_BWD, _p(gu), gu.stride(0), _p(ws), ws.numel(),
                         _stream()), "drl_gemm")
    return out


def linear_wgrad(gw, dy, x, accumulate=True, ws_slot=0):
    """gw (N_out, N_in) fp32 (+)= dy^T x (F.linear's grad_weight, accumulated in fp32): dy (T, N_out), x (T, N_in)."""
    T, M = dy.shape
    N = x.shape[1]
    assert x.shape[0] == T and gw.shape == (M, N) and gw.dtype == torch.float32
    return gemm(dy, LAYOUT_T, x, LAYOUT_T, M, N, T, gw, beta=accumulate, ws_slot=ws_slot)


_LINEAR_WS = {}


def _linear_workspace(device, nbytes, kind="linear"):
    """Per-device zeroed workspace shared by the split-K decode kernels of one kind on one stream (each call
    leaves its arrival tickets zeroed again, so consecutive calls and graph replays reuse it)."""
    key = (str(device), kind, _lane())
    ws = _LINEAR_WS.get(key)
    if ws is None or ws.numel() * 8 < nbytes:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError(f"{kind}: call once outside graph capture to size its workspace")
        ws = torch.zeros((max(nbytes, 1 << 22) + 7) // 8, dtype=torch.int64, device=device)
        _LINEAR_WS[key] = ws
    return ws


def decode_attention_vt(q, k_cache, vt_cache, key_valid, L, out, qpos=None, qpos_dev=None, out_mbt=0, group=1,
                        shared_keys=0):
    """MFMA decode attention: q (B,Hkv,G,D) bf16, k_cache (B,Hkv,ld_k,D), vt_cache (B,Hkv,D,ld_vt). ``out_mbt`` > 0:
    ``out`` is the fragment-packed (B, Hq*D) panel of the decode o_proj GEMM (decode_gemm layout). Prompt groups:
    rows p * group + r read keys < ``shared_keys`` (a multiple of 32) from cache row p."""
    _dev(q, k_cache, vt_cache, key_valid, out)
    B, Hkv, G, D = q.shape
    assert q.is_contiguous() and k_cache.is_contiguous() and out.is_contiguous()
    assert out_mbt == 0 or out.numel() >= out_mbt * 32 * Hkv * G * D
    assert key_valid.dtype == torch.uint8
    _vt_cap_ok(vt_cache, k_cache.shape[2])
    qp = L - 1 if qpos is None else int(qpos)
    nws = lib().drl_decode_attention_vt_workspace_bytes(B, Hkv, D, L)
    ws = _linear_workspace(q.device, nws, "decode_attention") if nws else None
    check(lib().drl_decode_attention_vt(_p(q), _p(k_cache), _p(vt_cache), _edt(q), _p(key_valid), key_valid.stride(0),
                                        _p(qpos_dev), qp, B, Hkv, G, D, k_cache.shape[2], vt_ld(vt_cache), L,
                                        int(group), int(shared_keys), 1.0 / math.sqrt(D), _p(out), int(out_mbt),
                                        _p(ws), nws, _stream()),
          "drl_decode_attention_vt")
    return out


def decode_step_prologue(responses, t_dev, t_cur, last_pos, prompt_len, embed, x, positions, kpos, key_valid,
                         x_mbt=0):
    """One launch of the graphed decode step's bookkeeping (drl_decode_step_prologue): x = float(embed[previous
    token]), positions = last_pos + t, key_valid[:, t + P - 1] = 1, kpos = t + P - 1, t_cur = t, t_dev += 1.
    ``x_mbt`` > 0: x is the fused-norm step's packed fp32 residual (x_mbt token blocks, flat)."""
    _dev(responses, t_dev, t_cur, last_pos, embed, x, positions, kpos, key_valid)
    assert responses.dtype == t_dev.dtype == t_cur.dtype == last_pos.dtype == positions.dtype == kpos.dtype == torch.int64
    assert embed.dtype == torch.bfloat16 and embed.is_contiguous() and x.dtype == torch.float32 and x.is_contiguous()
    assert key_valid.dtype == torch.uint8 and key_valid.stride(1) == 1 and responses.stride(1) == 1
    B, H = positions.numel(), embed.shape[1]
    assert x.numel() >= (x_mbt * 32 if x_mbt else B) * H
    V = embed.shape[0]
    assert last_pos.is_contiguous() and last_pos.numel() == B and positions.numel() == B and embed.shape[1] == H
    L = lib()
    ws = _linear_workspace(x.device, L.drl_decode_step_prologue_workspace_bytes(), "decode_prologue")
    check(L.drl_decode_step_prologue(_p(responses), responses.stride(0), _p(t_dev), _p(t_cur), _p(last_pos),
                                     int(prompt_len), _p(embed), _lib.DRL_BF16, V, H, B, _p(x), _p(positions), _p(kpos),
                                     _p(key_valid), key_valid.stride(0), _p(ws), ws.numel() * 8, int(x_mbt),
                                     _stream()),
          "drl_decode_step_prologue")


# ------------------------------------------------------------------------------ decode projections (packed)
DECODE_PARTIAL, DECODE_SWIGLU = 0, 1


def decode_gemm_plan(M, N, K, swiglu=False):
    """(ksplit, mbt) of drl_decode_gemm for this shape, or None when unsupported (K % 64, M > 128)."""
    ks, mbt = ctypes.c_int32(0), ctypes.c_int32(0)
    rc = lib().drl_decode_gemm_plan(M, N, K, DECODE_SWIGLU if swiglu else DECODE_PARTIAL, ctypes.byref(ks),
                                    ctypes.byref(mbt))
    return (ks.value, mbt.value) if rc == 0 else None


def decode_pack_weight(w, swiglu=False, out=None):
    """Fragment-packed copy of W (N, K) bf16 for drl_decode_gemm (swiglu: W = [gate | up])."""
    _dev(w)
    assert w.dim() == 2 and w.stride(1) == 1 and w.dtype == torch.bfloat16
    N, K = w.shape
    n = lib().drl_decode_pack_weight_elems(N, K, int(swiglu))
    if out is None:
        out = torch.empty(n, dtype=torch.bfloat16, device=w.device)
    assert out.numel() >= n and out.is_contiguous()
    check(lib().drl_decode_pack_weight(_p(w), w.stride(0), N, K, int(swiglu), _p(out), _stream()),
          "drl_decode_pack_weight")
    return out


def pack_activations(x, mbt):
    """Row-major (M, K) -> fragment-packed panel with mbt 32-row blocks (host-side layout helper for tests:
    element (m, k) at ((k//16 * mbt + m//32) * 64 + ((k//8) % 2) * 32 + m % 32) * 8 + k % 8)."""
    M, K = x.shape
    xp = torch.zeros(mbt * 32, K, dtype=x.dtype, device=x.device)
    xp[:M] = x
    return xp.view(mbt, 32, K // 16, 2, 8).permute(2, 0, 3, 1, 4).contiguous().view(-1)


def unpack_activations(xp, M, K, mbt):
    return xp.view(K // 16, mbt, 2, 32, 8).permute(1, 3, 0, 2, 4).reshape(mbt * 32, K)[:M]


def decode_gemm(x_packed, w_packed, M, N, K, swiglu=False, partials=None, out_packed=None):
    """x (packed, M rows) @ W^T (packed): fp32 partials (ksplit, M, N), or with ``swiglu`` the packed activation
    bf16(bf16(silu(g)) * u) (mbt blocks, N/2 columns)."""
    _dev(x_packed, w_packed)
    plan = decode_gemm_plan(M, N, K, swiglu)
    assert plan is not None, f"decode GEMM does not take M={M} N={N} K={K}"
    ks, mbt = plan
    assert x_packed.numel() >= mbt * 32 * K
    if swiglu:
        if out_packed is None:
            out_packed = torch.zeros(mbt * 32 * (N // 2), dtype=torch.bfloat16, device=x_packed.device)
    elif partials is None:
        partials = torch.empty(ks, M, N, dtype=torch.float32, device=x_packed.device)
    if swiglu:
        assert out_packed.numel() >= mbt * 32 * (N // 2) and out_packed.dtype == torch.bfloat16
    else:
        assert partials.numel() >= ks * M * N and partials.dtype == torch.float32 and partials.is_contiguous()
    check(lib().drl_decode_gemm(_p(x_packed), _p(w_packed), M, N, K, DECODE_SWIGLU if swiglu else DECODE_PARTIAL,
                                _p(partials), _p(out_packed), _stream()), "drl_decode_gemm")
    return out_packed if swiglu else partials


def decode_rmsnorm(x_in, partials, x_out, weight, y, eps, mbt=0, y_packed=None, packed_mbt=0):
    """x_out = x_in + bf16(sum partials); y = RMSNorm(x_out) * w in bf16, packed (mbt > 0) or row-major; with
    ``y_packed`` also written packed (packed_mbt blocks: the decode lm_head's operand)."""
    _dev(x_in, weight, y, y_packed)
    M, H = x_in.shape[0], x_in.shape[-1]
    ns = partials.shape[0] if partials is not None else 0
    check(lib().drl_decode_rmsnorm(_p(x_in), _p(partials), ns, _p(x_out), _p(weight), _p(y), M, H, int(mbt),
                                   float(eps), _p(y_packed), int(packed_mbt), _stream()), "drl_decode_rmsnorm")


def decode_rope(partials, bias, position_ids, cos_t, sin_t, Hq, Hkv, D, q, k_cache, vt_cache=None, v_cache=None,
                koff=0, koff_dev=None):
    """One decode token: qkv = bf16(sum partials + bias) -> RoPE -> q, k cache row koff, V^T / V cache."""
    _dev(partials, bias, position_ids, q, k_cache)
    ns, B = partials.shape[0], partials.shape[1]
    Tk = k_cache.shape[2]
    ld_vt = vt_ld(vt_cache) if vt_cache is not None else 0
    if vt_cache is not None:
        _vt_cap_ok(vt_cache, k_cache.shape[2])
    check(lib().drl_decode_rope(_p(partials), ns, _p(bias), _p(position_ids), _p(cos_t), _p(sin_t), cos_t.shape[0], B,
                                Hq, Hkv, D, _p(q), _p(k_cache), _p(v_cache), _p(vt_cache), Tk, ld_vt, int(koff),
                                _p(koff_dev), _stream()), "drl_decode_rope")


# ------------------------------------------------------------------------------ fused-norm decode step (ABI 8)
DECODE_RESID, DECODE_ROPE = 2, 3


def decode_norm_plan(M, N, K, epilogue):
    """(ksplit, mbt, config) of the fused-norm decode kernel for this shape (epilogue DECODE_RESID / DECODE_SWIGLU /
    DECODE_ROPE), or None when the shape takes the unfused step."""
    ks, mbt, cfg = ctypes.c_int32(0), ctypes.c_int32(0), ctypes.c_int32(0)
    rc = lib().drl_decode_norm_plan(M, N, K, epilogue, ctypes.byref(ks), ctypes.byref(mbt), ctypes.byref(cfg))
    return (ks.value, mbt.value, cfg.value) if rc == 0 else None


def decode_gemm_resid(x_packed, w_packed, M, N, K, x_resid, x_mbt, partials, counters):
    """o_proj / down_proj of the fused-norm step: x_resid (packed fp32) += bf16(x W^T) in place."""
    _dev(x_packed, w_packed, x_resid, partials, counters)
    assert x_resid.dtype == torch.float32 and x_resid.is_contiguous() and x_resid.numel() >= x_mbt * 32 * N
    assert partials is None or (partials.dtype == torch.float32 and partials.is_contiguous())
    nb = counters.numel() * counters.element_size() if counters is not None else 0
    check(lib().drl_decode_gemm_resid(_p(x_packed), _p(w_packed), M, N, K, _p(x_resid), int(x_mbt), _p(partials),
                                      _p(counters), nb, _stream()), "drl_decode_gemm_resid")


def decode_gemm_norm(x_resid, norm_weight, eps, w_packed, M, N, K, out_packed):
    """gate_up + SwiGLU of the fused-norm step on RMSNorm(x_resid) computed in the kernel's prologue."""
    _dev(x_resid, norm_weight, w_packed, out_packed)
    assert norm_weight.dtype == torch.float32 and norm_weight.is_contiguous() and norm_weight.numel() == K
    check(lib().drl_decode_gemm_norm(_p(x_resid), _p(norm_weight), float(eps), _p(w_packed), M, N, K, _p(out_packed),
                                     _stream()), "drl_decode_gemm_norm")
    return out_packed


def decode_qkv_rope_norm(x_resid, norm_weight, eps, w_packed, bias, position_ids, cos_t, sin_t, M, K, Hq, Hkv, D, q,
                         k_cache, vt_cache, koff_dev):
    """qkv + bias + RoPE + cache writes of the fused-norm step on RMSNorm(x_resid)."""
    _dev(x_resid, norm_weight, w_packed, bias, position_ids, q, k_cache, vt_cache, koff_dev)
    assert q.is_contiguous() and k_cache.is_contiguous() and norm_weight.dtype == torch.float32
    _vt_cap_ok(vt_cache, k_cache.shape[2])
    check(lib().drl_decode_qkv_rope_norm(_p(x_resid), _p(norm_weight), float(eps), _p(w_packed), _p(bias),
                                         _p(position_ids), _p(cos_t), _p(sin_t), cos_t.shape[0], M, K, Hq, Hkv, D, _p(q),
                                         _p(k_cache), _p(vt_cache), k_cache.shape[2], vt_ld(vt_cache), _p(koff_dev),
                                         _stream()), "drl_decode_qkv_rope_norm")


def decode_final_norm(x_resid, x_mbt, weight, y, M, H, eps, y_mbt=0, y_packed=None, packed_mbt=0):
    """The model's final RMSNorm from the packed fp32 residual: y bf16 row-major (M, H) or packed (y_mbt > 0), and
    optionally a second packed copy (y_packed, packed_mbt blocks)."""
    _dev(x_resid, weight, y, y_packed)
    check(lib().drl_decode_final_norm(_p(x_resid), int(x_mbt), _p(weight), _p(y), M, H, int(y_mbt), float(eps),
                                      _p(y_packed), int(packed_mbt), _stream()), "drl_decode_final_norm")
    return y


def decode_lm_head_plan(M, V, K):
    """Token blocks of the decode lm_head's packed operand, or None when the shape takes drl_gemm."""
    mbt = ctypes.c_int32(0)
    return mbt.value if lib().drl_decode_lm_head_plan(M, V, K, ctypes.byref(mbt)) == 0 else None


def decode_lm_head(h_packed, mbt, w_packed, M, V, K, out):
    """logits (M, V) bf16 = h W^T at <= 64 decode rows from the packed final-norm output (persistent kernel)."""
    _dev(h_packed, w_packed, out)
    assert out.dtype == torch.bfloat16 and out.stride(1) == 1 and out.shape == (M, V)
    check(lib().drl_decode_lm_head(_p(h_packed), int(mbt), _p(w_packed), M, V, K, _p(out), out.stride(0), _stream()),
          "drl_decode_lm_head")
    return out


def pack_residual(x, mbt, out=None):
    """Row-major fp32 (M, H) -> the fused-norm step's packed residual (mbt token blocks; rows >= M zero): element
    (m, k) at (((k//16 * mbt + m//32) * 2 + (k//4) % 2) * 64 + ((k//8) % 2) * 32 + m % 32) * 4 + k % 4."""
    M, H = x.shape
    xp = torch.zeros(mbt * 32, H, dtype=x.dtype, device=x.device)
    xp[:M] = x
    # (m_blk, m_in, k16, k8, k4, e) -> (k16, m_blk, k4, k8, m_in, e)
    xp = xp.view(mbt, 32, H // 16, 2, 2, 4).permute(2, 0, 4, 3, 1, 5).contiguous().view(-1)
    if out is None:
        return xp
    out.view(-1)[:xp.numel()].copy_(xp)
    return out


def unpack_residual(xp, M, H, mbt):
    return xp[:mbt * 32 * H].view(H // 16, mbt, 2, 2, 32, 4).permute(1, 4, 0, 3, 2, 5).reshape(mbt * 32, H)[:M]


def decode_pack_weight_rope(w, head_dim, out=None):
    """Packed qkv_proj weight in RoPE rotation pairs (drl_decode_qkv_rope)."""
    _dev(w)
    assert w.dim() == 2 and w.stride(1) == 1 and w.dtype == torch.bfloat16
    N, K = w.shape
    n = lib().drl_decode_pack_weight_elems(N, K, 0)
    if out is None:
        out = torch.empty(n, dtype=torch.bfloat16, device=w.device)
    check(lib().drl_decode_pack_weight_rope(_p(w), w.stride(0), N, K, head_dim, _p(out), _stream()),
          "drl_decode_pack_weight_rope")
    return out


def decode_qkv_rope(x_packed, w_packed, bias, position_ids, cos_t, sin_t, M, K, Hq, Hkv, D, q, k_cache, vt_cache,
                    koff_dev):
    """One launch: qkv_proj + bias + RoPE, q (M,Hkv,G,D) out, K / V^T cache rows at the device offset."""
    _dev(x_packed, w_packed, bias, position_ids, q, k_cache, vt_cache, koff_dev)
    assert q.is_contiguous() and k_cache.is_contiguous()
    _vt_cap_ok(vt_cache, k_cache.shape[2])
    check(lib().drl_decode_qkv_rope(_p(x_packed), _p(w_packed), _p(bias), _p(position_ids), _p(cos_t), _p(sin_t),
                                    cos_t.shape[0], M, K, Hq, Hkv, D, _p(q), _p(k_cache), _p(vt_cache),
                                    k_cache.shape[2], vt_ld(vt_cache), _p(koff_dev), _stream()),
          "drl_decode_qkv_rope")
