"""PPO/GRPO algorithm entry points with the reference's names and registries, computed by the HIP kernels.

Mirror of verl/trainer/ppo/core_algos.py (file:line per function). Registries and signatures are kept
so reference call sites and custom registrations map over unchanged; the numerics run in
libdotsrl_amd.so (K1 fused loss, K3 GRPO, K5 GAE).
"""

from __future__ import annotations

from collections.abc import Callable
from enum import Enum
from typing import Any

import numpy as np
import torch

from . import native

POLICY_LOSS_REGISTRY: dict[str, Callable] = {}
ADV_ESTIMATOR_REGISTRY: dict[str, Any] = {}


def register_policy_loss(name: str):
    """core_algos.py:51-66."""

    def decorator(func):
        POLICY_LOSS_REGISTRY[name] = func
        return func

    return decorator


def get_policy_loss_fn(name):
    """core_algos.py:69-83."""
    if name not in POLICY_LOSS_REGISTRY:
        raise ValueError(f"Unsupported loss mode: {name}. Supported modes are: {list(POLICY_LOSS_REGISTRY.keys())}")
    return POLICY_LOSS_REGISTRY[name]


class AdvantageEstimator(str, Enum):
    """core_algos.py:86-103."""

    GAE = "gae"
    GRPO = "grpo"
    REINFORCE_PLUS_PLUS = "reinforce_plus_plus"
    REINFORCE_PLUS_PLUS_BASELINE = "reinforce_plus_plus_baseline"
    REMAX = "remax"
    RLOO = "rloo"
    OPO = "opo"
    GRPO_PASSK = "grpo_passk"
    GPG = "gpg"


def register_adv_est(name_or_enum):
    """core_algos.py:109-126."""

    def decorator(fn):
        name = name_or_enum.value if isinstance(name_or_enum, Enum) else name_or_enum
        if name in ADV_ESTIMATOR_REGISTRY and ADV_ESTIMATOR_REGISTRY[name] != fn:
            raise ValueError(f"Adv estimator {name} has already been registered: {ADV_ESTIMATOR_REGISTRY[name]} vs {fn}")
        ADV_ESTIMATOR_REGISTRY[name] = fn
        return fn

    return decorator


def get_adv_estimator_fn(name_or_enum):
    """core_algos.py:129-143."""
    name = name_or_enum.value if isinstance(name_or_enum, Enum) else name_or_enum
    if name not in ADV_ESTIMATOR_REGISTRY:
        raise ValueError(f"Unknown advantage estimator simply: {name}")
    return ADV_ESTIMATOR_REGISTRY[name]


class AdaptiveKLController:
    """core_algos.py:146-170."""

    def __init__(self, init_kl_coef, target_kl, horizon):
        self.value = init_kl_coef
        self.target = target_kl
        self.horizon = horizon

    def update(self, current_kl, n_steps):
        proportional_error = np.clip(current_kl / self.target - 1, -0.2, 0.2)
        self.value *= 1 + proportional_error * n_steps / self.horizon


class FixedKLController:
    """core_algos.py:173-187."""

    def __init__(self, kl_coef):
        self.value = kl_coef

    def update(self, current_kl, n_steps):
        pass


def get_kl_controller(kl_ctrl):
    """core_algos.py:190-205."""
    if kl_ctrl.type == "fixed":
        return FixedKLController(kl_coef=kl_ctrl.kl_coef)
    if kl_ctrl.type == "adaptive":
        assert kl_ctrl.horizon > 0, f"horizon must be larger than 0. Got {kl_ctrl.horizon}"
        return AdaptiveKLController(init_kl_coef=kl_ctrl.kl_coef, target_kl=kl_ctrl.target_kl, horizon=kl_ctrl.horizon)
    raise NotImplementedError


# ---------------------------------------------------------------------------------------------- advantages
@register_adv_est(AdvantageEstimator.GAE)
def compute_gae_advantage_return(token_level_rewards, values, response_mask, gamma, lam):
    """core_algos.py:208-256 — HIP reverse scan + masked_whiten (K5)."""
    with torch.no_grad():
        return native.gae_advantage_return(token_level_rewards, values, response_mask, float(gamma), float(lam))


def uid_csr(index, device):
    """uid array -> (row_group[B], group_offsets[G+1], group_members[B], G): groups in order of first
    appearance, members in row order (the order core_algos.py:297-309 stacks them)."""
    keys = {}
    row_group = np.empty(len(index), np.int32)
    for i, u in enumerate(index):
        row_group[i] = keys.setdefault(u, len(keys))
    G = len(keys)
    members = np.argsort(row_group, kind="stable").astype(np.int32)
    offsets = np.zeros(G + 1, np.int32)
    np.add.at(offsets, row_group + 1, 1)
    offsets = np.cumsum(offsets).astype(np.int32)
    t = lambda a: torch.from_numpy(a).to(device, non_blocking=True)  # noqa: E731
    return t(row_group), t(offsets), t(members), G


@register_adv_est(AdvantageEstimator.GRPO)
def compute_grpo_outcome_advantage(token_level_rewards, response_mask, index, epsilon: float = 1e-6,
                                   norm_adv_by_std_in_grpo: bool = True, config=None):
    """core_algos.py:260-324 — scores, group mean/std and the (B, R) broadcast on device (K3)."""
    row_group, offsets, members, G = uid_csr(index, token_level_rewards.device)
    with torch.no_grad():
        return native.grpo_outcome_advantage(token_level_rewards, response_mask, row_group, offsets, members, G,
                                             epsilon, norm_adv_by_std_in_grpo)


@register_adv_est(AdvantageEstimator.RLOO)
def compute_rloo_outcome_advantage(token_level_rewards, response_mask, index, epsilon: float = 1e-6, config=None,
                                   **kwargs):
    """core_algos.py:444-493 — leave-one-out baseline per uid group (K3, RLOO mode)."""
    row_group, offsets, members, G = uid_csr(index, token_level_rewards.device)
    with torch.no_grad():
        return native.group_outcome_advantage("rloo", token_level_rewards, response_mask, row_group, offsets, members, G)


@register_adv_est(AdvantageEstimator.REINFORCE_PLUS_PLUS_BASELINE)
def compute_reinforce_plus_plus_baseline_outcome_advantage(token_level_rewards, response_mask, index,
                                                           epsilon: float = 1e-6, config=None, **kwargs):
    """core_algos.py:392-441 — group-mean baseline, then masked_whiten over the batch (K3 mode + whitening pass)."""
    row_group, offsets, members, G = uid_csr(index, token_level_rewards.device)
    with torch.no_grad():
        return native.group_outcome_advantage("reinforce_plus_plus_baseline", token_level_rewards, response_mask,
                                              row_group, offsets, members, G)


@register_adv_est(AdvantageEstimator.GRPO_PASSK)
def compute_grpo_passk_outcome_advantage(token_level_rewards, response_mask, index, epsilon: float = 1e-6,
                                         norm_adv_by_std_in_grpo: bool = True, config=None, **kwargs):
    """core_algos.py:327-386 — only the best sample of a uid group gets r_max - r_second_max (/ (std + eps)); K3
    pass@k mode. Groups of one sample raise, as the reference does."""
    assert config is not None
    norm = config.get("norm_adv_by_std_in_grpo", True)
    counts = {}
    for u in index:
        counts[u] = counts.get(u, 0) + 1
    for u, c in counts.items():
        if c < 2:
            raise ValueError(f"Pass@k requires at least 2 samples per group. Got {c} for group {u}.")
    row_group, offsets, members, G = uid_csr(index, token_level_rewards.device)
    with torch.no_grad():
        return native.group_outcome_advantage("grpo_passk", token_level_rewards, response_mask, row_group, offsets,
                                              members, G, epsilon, norm)


@register_adv_est(AdvantageEstimator.OPO)
def compute_opo_outcome_advantage(token_level_rewards, response_mask, index, epsilon: float = 1e-6, config=None,
                                  **kwargs):
    """core_algos.py:495-546 — score minus the length-weighted group mean (sum(len * s) / sum(len)); K3 OPO mode."""
    row_group, offsets, members, G = uid_csr(index, token_level_rewards.device)
    with torch.no_grad():
        return native.group_outcome_advantage("opo", token_level_rewards, response_mask, row_group, offsets, members, G)


@register_adv_est(AdvantageEstimator.GPG)
def compute_gpg_outcome_advantage(token_level_rewards, response_mask, index, epsilon: float = 1e-6, f_norm: float = 1.0,
                                  alpha: float = 1.0, config=None, **kwargs):
    """core_algos.py:624-684 — alpha * (s - group mean) / f_norm with alpha = B / max(#nonzero scores, 1) (the
    reference recomputes alpha and ignores the argument; f_norm = 1 as every caller passes); K3 GPG mode."""
    if f_norm != 1.0:
        raise NotImplementedError("GPG advantage with f_norm != 1")
    row_group, offsets, members, G = uid_csr(index, token_level_rewards.device)
    with torch.no_grad():
        return native.group_outcome_advantage("gpg", token_level_rewards, response_mask, row_group, offsets, members, G)


@register_adv_est(AdvantageEstimator.REMAX)
def compute_remax_outcome_advantage(token_level_rewards, reward_baselines, response_mask, config=None, **kwargs):
    """core_algos.py:588-621 — reverse cumsum of the masked rewards minus the greedy-rollout baseline score."""
    with torch.no_grad():
        return native.remax_advantage_return(token_level_rewards, reward_baselines, response_mask)


@register_adv_est(AdvantageEstimator.REINFORCE_PLUS_PLUS)
def compute_reinforce_plus_plus_outcome_advantage(token_level_rewards, response_mask, config=None, **kwargs):
    """core_algos.py:550-586 — masked discounted return scan + masked_whiten (K5 scan mode)."""
    assert config is not None
    with torch.no_grad():
        return native.reinforce_pp_advantage_return(token_level_rewards, response_mask, float(config.gamma))


# ---------------------------------------------------------------------------------------------- losses
def agg_loss(loss_mat, loss_mask, loss_agg_mode: str):
    """core_algos.py:703-736 (forward; gradients flow through fused_actor_loss)."""
    if loss_mat.requires_grad:
        raise NotImplementedError("differentiate the actor loss through fused_actor_loss (one HIP pass fwd+bwd)")
    return native.agg_loss(loss_mat, loss_mask, loss_agg_mode)


def kl_penalty(logprob, ref_logprob, kl_penalty):
    """core_algos.py:1272-1307 (forward; the KL gradient is part of fused_actor_loss)."""
    if kl_penalty == "full":
        raise NotImplementedError
    if logprob.requires_grad:
        raise NotImplementedError("differentiate the KL term through fused_actor_loss")
    return native.kl_penalty(logprob, ref_logprob, kl_penalty)


class _FusedActorLoss(torch.autograd.Function):
    """K1: forward AND backward computed in the forward launch; backward only scales the stored grads."""

    @staticmethod
    def forward(ctx, log_prob, entropy, old_log_prob, advantages, response_mask, ref_log_prob, kw):
        out, dlogp, dent = native.ppo_loss_fwd_bwd(
            old_log_prob.detach(), log_prob.detach(), advantages, response_mask,
            entropy.detach() if entropy is not None else None, ref_log_prob,
            want_dlogp=log_prob.requires_grad, want_dentropy=entropy is not None and entropy.requires_grad, **kw)
        ctx.save_for_backward(dlogp if dlogp is not None else out.new_empty(0),
                              dent if dent is not None else out.new_empty(0))
        ctx.has = (dlogp is not None, dent is not None)
        return out

    @staticmethod
    def backward(ctx, g):
        dlogp, dent = ctx.saved_tensors
        scale = g[6]  # only the total loss (DRL_PPO_OUT_LOSS) carries a gradient
        return (dlogp * scale if ctx.has[0] else None, dent * scale if ctx.has[1] else None,
                None, None, None, None, None)


def fused_actor_loss(log_prob, entropy, old_log_prob, advantages, response_mask, ref_log_prob, *, clip_ratio_low,
                     clip_ratio_high, clip_ratio_c, entropy_coeff, use_kl_loss, kl_loss_type, kl_loss_coef,
                     loss_agg_mode, loss_scale_factor, policy_loss="vanilla", cov_kw=None, token_count=None):
    """The whole per-micro-batch loss of dp_actor.py:419-466 in one HIP launch.

    Returns a float32[8] tensor: pg_loss, pg_clipfrac, ppo_kl, pg_clipfrac_lower, entropy_loss, kl_loss,
    loss (= (pg - c_ent*ent + c_kl*kl) * loss_scale_factor, the backpropagated value), mask_count.
    ``token_count`` (device float64 (1,), token-mean with the vanilla / gpg loss): sum(response_mask) of this
    micro-batch, computed by the caller for all micro-batches at once — K1 then reads the mask once (one pass).
    """
    kw = dict(clip_ratio_low=clip_ratio_low, clip_ratio_high=clip_ratio_high, clip_ratio_c=clip_ratio_c,
              entropy_coeff=entropy_coeff if entropy is not None else 0.0,
              kl_loss_coef=kl_loss_coef if use_kl_loss else 0.0,
              kl_loss_type=kl_loss_type if use_kl_loss else None, loss_agg_mode=loss_agg_mode,
              loss_scale_factor=loss_scale_factor, policy_loss=policy_loss, **(cov_kw or {}))
    if token_count is not None and loss_agg_mode == "token-mean" and policy_loss in ("vanilla", "gpg"):
        kw["token_count"] = token_count
    return _FusedActorLoss.apply(log_prob, entropy, old_log_prob, advantages, response_mask,
                                 ref_log_prob if use_kl_loss else None, kw)


@register_policy_loss("vanilla")
def compute_policy_loss_vanilla(old_log_prob, log_prob, advantages, response_mask, loss_agg_mode: str = "token-mean",
                                config=None):
    """core_algos.py:815-889 — (pg_loss, pg_clipfrac, ppo_kl, pg_clipfrac_lower); pg_loss is differentiable."""
    assert config is not None
    clip_ratio = config.clip_ratio
    lo = config.clip_ratio_low if config.get("clip_ratio_low") is not None else clip_ratio
    hi = config.clip_ratio_high if config.get("clip_ratio_high") is not None else clip_ratio
    c = config.get("clip_ratio_c", 3.0)
    assert c > 1.0, ("The lower bound of the clip_ratio_c for dual-clip PPO should be greater than 1.0,"
                     + f" but get the value: {c}.")
    out = fused_actor_loss(log_prob, None, old_log_prob, advantages, response_mask, None, clip_ratio_low=lo,
                           clip_ratio_high=hi, clip_ratio_c=c, entropy_coeff=0.0, use_kl_loss=False,
                           kl_loss_type=None, kl_loss_coef=0.0, loss_agg_mode=loss_agg_mode, loss_scale_factor=1.0)
    # out[6] == pg_loss here (no entropy / KL term, scale 1) and is the differentiable slot
    return out[6], out[1].detach(), out[2].detach(), out[3].detach()


@register_policy_loss("gpg")
def compute_policy_loss_gpg(old_log_prob, log_prob, advantages, response_mask, loss_agg_mode="token-mean", config=None):
    """core_algos.py:957-975 — pg = -log_prob * advantages (K1, GPG mode); clip metrics are 0."""
    out = fused_actor_loss(log_prob, None, old_log_prob, advantages, response_mask, None, clip_ratio_low=0.2,
                           clip_ratio_high=0.2, clip_ratio_c=3.0, entropy_coeff=0.0, use_kl_loss=False,
                           kl_loss_type=None, kl_loss_coef=0.0, loss_agg_mode=loss_agg_mode, loss_scale_factor=1.0,
                           policy_loss="gpg")
    return out[6], out[1].detach(), out[2].detach(), out[3].detach()


def _clip_lo_hi(config):
    lo = config.clip_ratio_low if config.get("clip_ratio_low") is not None else config.clip_ratio
    hi = config.clip_ratio_high if config.get("clip_ratio_high") is not None else config.clip_ratio
    return lo, hi


@register_policy_loss("gspo")
def compute_policy_loss_gspo(old_log_prob, log_prob, advantages, response_mask, loss_agg_mode="seq-mean-token-mean",
                             config=None):
    """core_algos.py:892-954 — sequence-level importance ratio, PPO clip, seq-mean-token-mean (K1's GSPO path)."""
    assert config is not None
    lo, hi = _clip_lo_hi(config)
    out = fused_actor_loss(log_prob, None, old_log_prob, advantages, response_mask, None, clip_ratio_low=lo,
                           clip_ratio_high=hi, clip_ratio_c=3.0, entropy_coeff=0.0, use_kl_loss=False,
                           kl_loss_type=None, kl_loss_coef=0.0, loss_agg_mode=loss_agg_mode, loss_scale_factor=1.0,
                           policy_loss="gspo")
    return out[6], out[1].detach(), out[2].detach(), out[3].detach()


@register_policy_loss("geo_mean")
def compute_policy_loss_geo_mean(old_log_prob, log_prob, advantages, response_mask, loss_agg_mode="token-mean",
                                 config=None):
    """core_algos.py:1143-1210 — GMPO geometric-mean ratio per sequence (K1's GMPO path); loss_agg_mode unused."""
    assert config is not None
    lo, hi = _clip_lo_hi(config)
    out = fused_actor_loss(log_prob, None, old_log_prob, advantages, response_mask, None, clip_ratio_low=lo,
                           clip_ratio_high=hi, clip_ratio_c=3.0, entropy_coeff=0.0, use_kl_loss=False,
                           kl_loss_type=None, kl_loss_coef=0.0, loss_agg_mode=loss_agg_mode, loss_scale_factor=1.0,
                           policy_loss="geo_mean")
    return out[6], out[1].detach(), out[2].detach(), out[3].detach()


_COV_SEED = [0]


def _mix64(x):
    """splitmix64 finaliser (a fixed bijection of 64-bit words)."""
    x = (x + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return x ^ (x >> 31)


def cov_loss_kw(policy_loss_cfg, mode, seed_key=None):
    """clip_cov / kl_cov knobs from actor.policy_loss (PolicyLossConfig defaults, workers/config/actor.py:45-50) and
    the clip_cov subset seed. The reference draws the subset from torch's global RNG, whose state its checkpoint
    restores; here the seed is a function of ``seed_key`` = (policy_loss.seed, optimizer step, micro-batch index),
    all of which a checkpoint restores, so a resumed run draws the same subsets as an uninterrupted one. Without a
    key (direct registry calls) a per-process call counter stands in."""
    pc = policy_loss_cfg or {}
    get = (lambda k, d: pc.get(k) if pc.get(k) is not None else d)
    if seed_key is None:
        _COV_SEED[0] += 1
        seed_key = (0x5EED, _COV_SEED[0])
    seed = 0
    for part in seed_key:
        seed = _mix64(seed ^ (int(part) & 0xFFFFFFFFFFFFFFFF))
    ratio = get("clip_cov_ratio", 0.0002) if mode == "clip_cov" else get("kl_cov_ratio", 0.0002)
    return dict(cov_ratio=ratio, clip_cov_lb=get("clip_cov_lb", 1.0), clip_cov_ub=get("clip_cov_ub", 5.0),
                ppo_kl_coef=get("ppo_kl_coef", 0.1), cov_seed=seed)


@register_policy_loss("clip_cov")
def compute_policy_loss_clip_cov(old_log_prob, log_prob, advantages, response_mask, loss_agg_mode="token-mean",
                                 config=None):
    """core_algos.py:978-1069 — PPO clip with the loss of a random subset of high-covariance tokens zeroed (K1's
    covariance path; the subset is our seeded draw, see include/dotsrl_amd.h)."""
    assert config is not None and config.get("policy_loss") is not None
    lo, hi = _clip_lo_hi(config)
    out = fused_actor_loss(log_prob, None, old_log_prob, advantages, response_mask, None, clip_ratio_low=lo,
                           clip_ratio_high=hi, clip_ratio_c=3.0, entropy_coeff=0.0, use_kl_loss=False,
                           kl_loss_type=None, kl_loss_coef=0.0, loss_agg_mode=loss_agg_mode, loss_scale_factor=1.0,
                           policy_loss="clip_cov", cov_kw=cov_loss_kw(config.policy_loss, "clip_cov"))
    return out[6], out[1].detach(), out[2].detach(), out[3].detach()


@register_policy_loss("kl_cov")
def compute_policy_loss_kl_cov(old_log_prob, log_prob, advantages, response_mask, loss_agg_mode="token-mean",
                               config=None):
    """core_algos.py:1072-1140 — -A r, plus ppo_kl_coef |log_prob - old| on the top-k covariance tokens (K1's
    covariance path)."""
    assert config is not None and config.get("policy_loss") is not None
    out = fused_actor_loss(log_prob, None, old_log_prob, advantages, response_mask, None, clip_ratio_low=0.2,
                           clip_ratio_high=0.2, clip_ratio_c=3.0, entropy_coeff=0.0, use_kl_loss=False,
                           kl_loss_type=None, kl_loss_coef=0.0, loss_agg_mode=loss_agg_mode, loss_scale_factor=1.0,
                           policy_loss="kl_cov", cov_kw=cov_loss_kw(config.policy_loss, "kl_cov"))
    return out[6], out[1].detach(), out[2].detach(), out[3].detach()


def compute_value_loss(vpreds, returns, values, response_mask, cliprange_value, loss_agg_mode="token-mean"):
    """core_algos.py:1230-1269 — (vf_loss, vf_clipfrac); vf_loss is differentiable wrt vpreds (K6, one launch
    for forward and backward, csrc/value_loss.hip)."""
    from .dp_critic import fused_value_loss

    if loss_agg_mode not in ("token-mean", "seq-mean-token-sum", "seq-mean-token-mean", "seq-mean-token-sum-norm"):
        raise ValueError(f"Invalid loss_agg_mode: {loss_agg_mode}")
    out = fused_value_loss(vpreds, values, returns, response_mask, cliprange_value=cliprange_value,
                           loss_agg_mode=loss_agg_mode, loss_scale_factor=1.0)
    return out[3], out[1].detach()
