"""Numpy restatement of the reference hot-path math (TEST INFRASTRUCTURE — see oracle/__init__.py).

Each function cites the reference file:line (under /root/reference) it restates. Values are computed in
float64 from float32 inputs unless the reference's result depends on float32 rounding, so the oracle is
at least as accurate as the reference; forward values and analytic gradients are both given so the
HIP kernels' forward AND backward can be checked without autograd.
"""

from __future__ import annotations

import numpy as np

AGG_MODES = ("token-mean", "seq-mean-token-sum", "seq-mean-token-mean", "seq-mean-token-sum-norm")
KL_TYPES = {"kl": "k1", "k1": "k1", "abs": "abs", "mse": "k2", "k2": "k2", "low_var_kl": "k3", "k3": "k3"}

f64 = np.float64


# ---------------------------------------------------------------------------------------------
# masked reductions — verl/utils/torch_functional.py:163-223
# ---------------------------------------------------------------------------------------------
def masked_sum(values, mask, axis=None):
    """torch_functional.py:163-168: where(mask, v, 0) * mask, then sum."""
    v = np.where(np.asarray(mask).astype(bool), np.asarray(values, f64), 0.0)
    return (v * np.asarray(mask, f64)).sum(axis=axis)


def masked_mean(values, mask, axis=None):
    """torch_functional.py:171-185: masked_sum / (mask.sum() + 1e-8)."""
    return masked_sum(values, mask, axis) / (np.asarray(mask, f64).sum(axis=axis) + 1e-8)


def masked_var(values, mask, unbiased=True):
    """torch_functional.py:188-203 (raises on mask_sum in {0, 1} like the reference)."""
    mean = masked_mean(values, mask)
    var = masked_mean((np.asarray(values, f64) - mean) ** 2, mask)
    if unbiased:
        n = np.asarray(mask, f64).sum()
        if n == 0:
            raise ValueError("At least one element in the mask has to be 1.")
        if n == 1:
            raise ValueError("The sum of the mask is one, which can cause a division by zero.")
        var = var * (n / (n - 1))
    return var


def masked_whiten(values, mask, shift_mean=True):
    """torch_functional.py:206-223."""
    mean, var = masked_mean(values, mask), masked_var(values, mask)
    w = (np.asarray(values, f64) - mean) / np.sqrt(var + 1e-8)
    return w + mean if not shift_mean else w


# ---------------------------------------------------------------------------------------------
# agg_loss — verl/trainer/ppo/core_algos.py:703-736 (forward value and d loss / d loss_mat)
# ---------------------------------------------------------------------------------------------
def agg_loss(loss_mat, loss_mask, loss_agg_mode):
    x = np.asarray(loss_mat, f64)
    m = np.asarray(loss_mask, f64)
    B, R = x.shape
    with np.errstate(divide="ignore", invalid="ignore"):
        if loss_agg_mode == "token-mean":
            return masked_mean(x, loss_mask)
        if loss_agg_mode == "seq-mean-token-sum":
            return (x * m).sum(-1).mean()
        if loss_agg_mode == "seq-mean-token-mean":
            return ((x * m).sum(-1) / m.sum(-1)).mean()
        if loss_agg_mode == "seq-mean-token-sum-norm":
            return (x * m).sum(-1).sum() / R
    raise ValueError(f"Invalid loss_agg_mode: {loss_agg_mode}")


def agg_loss_grad(loss_mask, loss_agg_mode):
    """d agg_loss / d loss_mat (the same weights every reduction in agg_loss applies)."""
    m = np.asarray(loss_mask, f64)
    B, R = m.shape
    with np.errstate(divide="ignore", invalid="ignore"):
        if loss_agg_mode == "token-mean":
            return m / (m.sum() + 1e-8)
        if loss_agg_mode == "seq-mean-token-sum":
            return m / B
        if loss_agg_mode == "seq-mean-token-mean":
            return m / (B * m.sum(-1, keepdims=True))
        if loss_agg_mode == "seq-mean-token-sum-norm":
            return m / R
    raise ValueError(f"Invalid loss_agg_mode: {loss_agg_mode}")


# ---------------------------------------------------------------------------------------------
# kl_penalty — core_algos.py:1272-1307 (value and d/d logprob)
# ---------------------------------------------------------------------------------------------
def kl_penalty(logprob, ref_logprob, kl_penalty):
    kind = KL_TYPES.get(kl_penalty)
    lp = np.asarray(logprob, np.float32)
    rf = np.asarray(ref_logprob, np.float32)
    if kind == "k1":
        return (lp - rf).astype(f64), np.ones_like(lp, f64)
    if kind == "abs":
        d = lp - rf
        return np.abs(d).astype(f64), np.sign(d).astype(f64)
    if kind == "k2":
        d = (lp - rf).astype(f64)
        return 0.5 * d * d, d
    if kind == "k3":
        raw = (rf - lp).astype(f64)
        kl = np.clip(raw, -20.0, 20.0)
        g1 = ((raw >= -20.0) & (raw <= 20.0)).astype(f64)
        ratio = np.exp(kl)
        kld = ratio - kl - 1.0
        out = np.clip(kld, -10.0, 10.0)
        g2 = ((kld >= -10.0) & (kld <= 10.0)).astype(f64)
        return out, -(ratio - 1.0) * g1 * g2
    raise NotImplementedError(kl_penalty)


# ---------------------------------------------------------------------------------------------
# compute_policy_loss_vanilla — core_algos.py:815-889 (forward + analytic backward)
# ---------------------------------------------------------------------------------------------
def _max_grad(a, b):
    """torch.maximum backward (tools/autograd/derivatives.yaml): ties split the gradient in half."""
    ga = np.where(a > b, 1.0, np.where(a == b, 0.5, 0.0))
    return ga, 1.0 - ga


def policy_loss_vanilla(old_log_prob, log_prob, advantages, response_mask, loss_agg_mode="token-mean",
                        clip_ratio_low=0.2, clip_ratio_high=0.2, clip_ratio_c=3.0):
    """Returns (pg_loss, pg_clipfrac, ppo_kl, pg_clipfrac_lower, pg_losses, d pg_losses / d log_prob)."""
    assert clip_ratio_c > 1.0
    f32 = np.float32
    # per-token values in float32 with the reference's op order: the branch decisions (clip, ties,
    # clipfrac counts) depend on float32 rounding exactly at the clip bounds
    raw = np.asarray(log_prob, f32) - np.asarray(old_log_prob, f32)
    nkl = np.clip(raw, f32(-20.0), f32(20.0))
    gate = ((raw >= -20.0) & (raw <= 20.0)).astype(f64)
    ratio = np.exp(nkl.astype(f64)).astype(f32)  # correctly rounded float32 exp
    A = np.asarray(advantages, f32)
    negA = -A
    L1 = negA * ratio
    lo, hi = f32(1.0 - clip_ratio_low), f32(1.0 + clip_ratio_high)
    rc = np.clip(ratio, lo, hi)
    gc = ((ratio >= lo) & (ratio <= hi)).astype(f64)
    L2 = negA * rc
    C1 = np.maximum(L1, L2)
    w1, w2 = _max_grad(L1, L2)
    dC1 = w1 * (-A.astype(f64)) + w2 * (-A.astype(f64)) * gc
    L3 = negA * f32(clip_ratio_c)
    C2 = np.minimum(L3, C1)
    _, wc1 = _max_grad(-L3, -C1)  # min(a, b) backward == max(-a, -b) backward
    neg = A < 0
    pg_losses = np.where(neg, C2, C1).astype(f64)
    dpg_dratio = np.where(neg, wc1 * dC1, dC1)
    dpg = dpg_dratio * ratio.astype(f64) * gate
    nkl = nkl.astype(f64)
    m = response_mask
    pg_loss = agg_loss(pg_losses, m, loss_agg_mode)
    ppo_kl = masked_mean(-nkl, m)
    pg_clipfrac = masked_mean((L2 > L1).astype(f64), m)
    pg_clipfrac_lower = masked_mean((C1 > L3).astype(f64) * neg.astype(f64), m)
    return pg_loss, pg_clipfrac, ppo_kl, pg_clipfrac_lower, pg_losses, dpg


def clip_boundary_tokens(old_log_prob, log_prob, advantages, response_mask, clip_ratio_low=0.2, clip_ratio_high=0.2,
                         clip_ratio_c=3.0, ulps=2):
    """Masked tokens whose clip decisions hinge on the last ulp of exp (|ratio - bound| <= ulps ulp).

    float32 exp is not correctly rounded in torch (SLEEF), numpy or ocml, so pg_clipfrac and
    pg_clipfrac_lower may differ by one count per such token between any two implementations; the
    loss value and its gradient are continuous there and do not."""
    f32 = np.float32
    nkl = np.clip(np.asarray(log_prob, f32) - np.asarray(old_log_prob, f32), f32(-20), f32(20))
    ratio = np.exp(nkl.astype(f64))
    m = np.asarray(response_mask).astype(bool)
    amb = np.zeros_like(m)
    for bound in (f32(1.0 - clip_ratio_low), f32(1.0 + clip_ratio_high)):
        amb |= np.abs(ratio - f64(bound)) <= ulps * np.spacing(bound)
    A = np.asarray(advantages, f32)
    # C1 vs L3 = -A*c ties: ratio near c on the dual-clip side
    amb |= np.abs(ratio - f64(f32(clip_ratio_c))) <= ulps * np.spacing(f32(clip_ratio_c))
    amb |= A == 0
    return int((amb & m).sum())


def policy_loss_gspo(old_log_prob, log_prob, advantages, response_mask, clip_ratio_low=0.2, clip_ratio_high=0.2):
    """compute_policy_loss_gspo (core_algos.py:892-954): the sequence-mean log-ratio (length clamped at 1) as every
    token's log importance ratio (clamped at 10; d/d log_prob through the log_prob - sg(log_prob) term), PPO clip
    without dual clip, pg aggregated seq-mean-token-mean whatever loss_agg_mode says. Returns (pg_loss,
    pg_clipfrac, ppo_kl, pg_clipfrac_lower, d pg_loss / d log_prob)."""
    f32 = np.float32
    m32 = np.asarray(response_mask, f32)
    nak = np.asarray(log_prob, f32) - np.asarray(old_log_prob, f32)
    seq_len = np.maximum(m32.sum(-1), f32(1.0))
    seq_kl = ((nak * m32).sum(-1) / seq_len).astype(f32)
    lsr = np.minimum(seq_kl, f32(10.0))[:, None] * np.ones_like(nak)
    gate = (seq_kl <= 10.0)[:, None].astype(f64)
    ratio = np.exp(lsr.astype(f64)).astype(f32)
    A = np.asarray(advantages, f32)
    L1 = -A * ratio
    lo, hi = f32(1.0 - clip_ratio_low), f32(1.0 + clip_ratio_high)
    gc = ((ratio >= lo) & (ratio <= hi)).astype(f64)
    L2 = -A * np.clip(ratio, lo, hi)
    w1, w2 = _max_grad(L1, L2)
    dpg = (w1 + w2 * gc) * (-A.astype(f64)) * ratio.astype(f64) * gate
    pg_losses = np.maximum(L1, L2).astype(f64)
    mode = "seq-mean-token-mean"
    pg_loss = agg_loss(pg_losses, response_mask, mode)
    dpg = dpg * agg_loss_grad(response_mask, mode)
    return (pg_loss, masked_mean((L2 > L1).astype(f64), response_mask), masked_mean(-nak.astype(f64), response_mask),
            0.0, dpg)


def policy_loss_geo_mean(old_log_prob, log_prob, advantages, response_mask, clip_ratio_low=0.2, clip_ratio_high=0.2):
    """compute_policy_loss_geo_mean (core_algos.py:1143-1210, GMPO): token log-ratios clipped toward the advantage's
    sign (clamp to [-clip_ratio_low, clip_ratio_high] in log space, min under sign(A)), the row's geometric-mean
    ratio exp(mean over the row), the row's mean advantage, pg = mean over rows of -adv * ratio. Returns (pg_loss,
    pg_clipfrac, ppo_kl, pg_clipfrac_lower, d pg_loss / d log_prob)."""
    f32 = np.float32
    m32 = np.asarray(response_mask, f32)
    nak = np.asarray(log_prob, f32) - np.asarray(old_log_prob, f32)
    A = np.asarray(advantages, f32)
    sgn = np.sign(A)
    lo, hi = f32(clip_ratio_low), f32(clip_ratio_high)
    ncl = np.clip(nak, -lo, hi)
    gc = ((nak >= -lo) & (nak <= hi)).astype(f64)
    a, b = sgn * nak, sgn * ncl
    wa, wb = _max_grad(-a, -b)  # min backward
    nmin = sgn * np.minimum(a, b)
    dnmin = (sgn.astype(f64) ** 2) * (wa + wb * gc)
    msum = m32.sum(-1) + f32(1e-8)
    ratio = np.exp(((nmin * m32).sum(-1) / msum).astype(f64)).astype(f32)
    adv = ((A * m32).sum(-1) / msum).astype(f32)
    pg_rows = (-adv * ratio).astype(f64)
    B = A.shape[0]
    pg_loss = pg_rows.mean()
    dpg = ((-adv.astype(f64) * ratio.astype(f64) / msum.astype(f64)) / B)[:, None] * m32.astype(f64) * dnmin
    clipped = (nak != ncl).astype(f64)
    return (pg_loss, masked_mean(clipped * (A > 0), response_mask), masked_mean(-nak.astype(f64), response_mask),
            masked_mean(clipped * (A < 0), response_mask), dpg)


def fmix32(x):
    """murmur3's 32-bit finalizer (a bijection), vectorised over uint32 — clip_cov's subset ranking."""
    h = np.asarray(x, np.uint64) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(16)
    h = (h * np.uint64(0x85EBCA6B)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(13)
    h = (h * np.uint64(0xC2B2AE35)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(16)
    return h.astype(np.uint32)


def policy_loss_kl_cov(old_log_prob, log_prob, advantages, response_mask, loss_agg_mode="token-mean",
                       kl_cov_ratio=0.0002, ppo_kl_coef=0.1):
    """compute_policy_loss_kl_cov (core_algos.py:1072-1140): pg = -A r (r = exp(log_prob - old), unclamped), plus
    ppo_kl_coef |log_prob - old| on the max(1, int(n_valid * kl_cov_ratio)) valid tokens with the largest
    covariance (A - mean A)(log_prob - mean log_prob) (means over the valid tokens; equal values: lowest flat index
    first). Returns (pg_loss, 0, ppo_kl = masked_mean(|nak|), 0, d pg_loss / d log_prob)."""
    f32 = np.float32
    nak = np.asarray(log_prob, f32) - np.asarray(old_log_prob, f32)
    r = np.exp(nak.astype(f64)).astype(f32)
    A = np.asarray(advantages, f32)
    lp = np.asarray(log_prob, f32)
    valid = np.asarray(response_mask) > 0
    pg = (-A * r).astype(f64)
    dpg = (-A * r).astype(f64)
    n = int(valid.sum())
    if n > 0:
        ma = f32(A[valid].astype(f64).mean())
        ml = f32(lp[valid].astype(f64).mean())
        flat = np.flatnonzero(valid.reshape(-1))
        cov = ((A.reshape(-1)[flat] - ma) * (lp.reshape(-1)[flat] - ml)).astype(f32)
        k = max(1, int(n * kl_cov_ratio))
        pick = flat[np.argsort(-cov.astype(f64), kind="stable")[:k]]
        nk = nak.reshape(-1)
        pg.reshape(-1)[pick] += ppo_kl_coef * np.abs(nk[pick])
        dpg.reshape(-1)[pick] += ppo_kl_coef * np.sign(nk[pick])
    pg_loss = agg_loss(pg, response_mask, loss_agg_mode)
    return pg_loss, 0.0, masked_mean(np.abs(nak).astype(f64), response_mask), 0.0, \
        dpg * agg_loss_grad(response_mask, loss_agg_mode)


def policy_loss_clip_cov(old_log_prob, log_prob, advantages, response_mask, loss_agg_mode="token-mean",
                         clip_ratio_low=0.2, clip_ratio_high=0.2, clip_cov_ratio=0.0002, clip_cov_lb=1.0,
                         clip_cov_ub=5.0, cov_seed=0, return_selected=False):
    """compute_policy_loss_clip_cov (core_algos.py:978-1069): PPO clip (no dual clip) with corr = 0 on
    min(clip_num, #candidates) candidates (valid, not clipped by the PPO clip, lb < cov < ub; cov with masked means),
    clip_num = max(int(clip_cov_ratio * sum(mask)), 1). The reference draws the subset with torch.randperm; the HIP
    path (and this restatement) takes the candidates with the smallest fmix32(flat index ^ seed32) — the same
    result whenever every candidate fits. Returns (pg_loss, pg_clipfrac, ppo_kl, 0, d pg_loss / d log_prob)."""
    f32 = np.float32
    nak = np.asarray(log_prob, f32) - np.asarray(old_log_prob, f32)
    r = np.exp(nak.astype(f64)).astype(f32)
    A = np.asarray(advantages, f32)
    lp = np.asarray(log_prob, f32)
    m32 = np.asarray(response_mask, f32)
    L1 = -A * r
    lo, hi = f32(1.0 - clip_ratio_low), f32(1.0 + clip_ratio_high)
    L2 = -A * np.clip(r, lo, hi)
    gc = ((r >= lo) & (r <= hi)).astype(f64)
    msum = m32.sum()
    ma = f32((A * m32).sum() / (msum + f32(1e-8)))
    ml = f32((lp * m32).sum() / (msum + f32(1e-8)))
    cov = ((A - ma) * (lp - ml)).astype(f32)
    cand = (m32 > 0) & ~(L2 > L1) & (cov < f32(clip_cov_ub)) & (cov > f32(clip_cov_lb))
    clip_num = max(int(clip_cov_ratio * float(msum)), 1)
    flat = np.flatnonzero(cand.reshape(-1))
    if len(flat) > clip_num:
        seed32 = (cov_seed ^ (cov_seed >> 32)) & 0xFFFFFFFF
        flat = flat[np.argsort(fmix32(flat.astype(np.uint64) ^ np.uint64(seed32)), kind="stable")[:clip_num]]
    sel = np.zeros(A.size, bool)
    sel[flat] = True
    sel = sel.reshape(A.shape)
    corr = (~sel).astype(f64)
    w1, w2 = _max_grad(L1, L2)
    pg = np.maximum(L1, L2).astype(f64) * corr
    dpg = corr * (w1 + w2 * gc) * (-A.astype(f64)) * r.astype(f64)
    pg_loss = agg_loss(pg, response_mask, loss_agg_mode)
    out = (pg_loss, masked_mean(sel.astype(f64), response_mask), masked_mean(-nak.astype(f64), response_mask), 0.0,
           dpg * agg_loss_grad(response_mask, loss_agg_mode))
    return out + (sel,) if return_selected else out


def actor_loss(old_log_prob, log_prob, advantages, response_mask, entropy, ref_log_prob, *, loss_agg_mode,
               clip_ratio_low, clip_ratio_high, clip_ratio_c, entropy_coeff, use_kl_loss, kl_loss_type,
               kl_loss_coef, loss_scale_factor, policy_loss="vanilla", cov_ratio=0.0002, clip_cov_lb=1.0,
               clip_cov_ub=5.0, ppo_kl_coef=0.1, cov_seed=0):
    """The per-micro-batch loss of DataParallelPPOActor.update_policy (dp_actor.py:419-466).
    policy_loss "gpg": compute_policy_loss_gpg (core_algos.py:957-975), pg = -log_prob * advantages; "gspo" /
    "geo_mean": policy_loss_gspo / policy_loss_geo_mean (sequence-level ratios)."""
    w = agg_loss_grad(response_mask, loss_agg_mode)
    if policy_loss in ("gspo", "geo_mean", "clip_cov", "kl_cov"):  # the pg gradient carries its own agg weights
        if policy_loss == "kl_cov":
            pg_loss, clipfrac, ppo_kl, clipfrac_lower, dpg_w = policy_loss_kl_cov(
                old_log_prob, log_prob, advantages, response_mask, loss_agg_mode, cov_ratio, ppo_kl_coef)
        elif policy_loss == "clip_cov":
            pg_loss, clipfrac, ppo_kl, clipfrac_lower, dpg_w = policy_loss_clip_cov(
                old_log_prob, log_prob, advantages, response_mask, loss_agg_mode, clip_ratio_low, clip_ratio_high,
                cov_ratio, clip_cov_lb, clip_cov_ub, cov_seed)
        else:
            fn = policy_loss_gspo if policy_loss == "gspo" else policy_loss_geo_mean
            pg_loss, clipfrac, ppo_kl, clipfrac_lower, dpg_w = fn(old_log_prob, log_prob, advantages, response_mask,
                                                                   clip_ratio_low, clip_ratio_high)
        with np.errstate(divide="ignore", invalid="ignore"):
            dpg = np.where(w != 0, dpg_w / np.where(w != 0, w, 1.0), 0.0)
    elif policy_loss == "gpg":
        lp32 = np.asarray(log_prob, np.float32)
        A32 = np.asarray(advantages, np.float32)
        pg_losses = ((-lp32) * A32).astype(f64)
        pg_loss = agg_loss(pg_losses, response_mask, loss_agg_mode)
        clipfrac = ppo_kl = clipfrac_lower = 0.0
        dpg = -A32.astype(f64)
    else:
        pg_loss, clipfrac, ppo_kl, clipfrac_lower, _, dpg = policy_loss_vanilla(
            old_log_prob, log_prob, advantages, response_mask, loss_agg_mode, clip_ratio_low, clip_ratio_high,
            clip_ratio_c)
    entropy_loss = agg_loss(entropy, response_mask, loss_agg_mode)
    total = pg_loss - entropy_loss * entropy_coeff if entropy_coeff != 0 else pg_loss
    kld, dkld = kl_penalty(log_prob, ref_log_prob, kl_loss_type)
    kl_loss = agg_loss(kld, response_mask, loss_agg_mode)
    dlogp = dpg_w if policy_loss in ("gspo", "geo_mean", "clip_cov", "kl_cov") else w * dpg
    if use_kl_loss:
        total = total + kl_loss * kl_loss_coef
        dlogp = dlogp + kl_loss_coef * w * dkld
    dent = -entropy_coeff * w if entropy_coeff != 0 else np.zeros_like(w)
    return dict(pg_loss=pg_loss, pg_clipfrac=clipfrac, ppo_kl=ppo_kl, pg_clipfrac_lower=clipfrac_lower,
                entropy_loss=entropy_loss, kl_loss=kl_loss, loss=total * loss_scale_factor,
                dlogp=dlogp * loss_scale_factor, dentropy=dent * loss_scale_factor, kld=kld)


# ---------------------------------------------------------------------------------------------
# compute_grpo_outcome_advantage — core_algos.py:260-324
# ---------------------------------------------------------------------------------------------
def grpo_outcome_advantage(token_level_rewards, response_mask, index, epsilon=1e-6, norm_adv_by_std_in_grpo=True):
    r = np.asarray(token_level_rewards, np.float32)
    scores = r.astype(f64).sum(-1)
    groups: dict = {}
    for i, u in enumerate(index):
        groups.setdefault(u, []).append(i)
    out = np.empty_like(scores)
    for members in groups.values():
        s = scores[members]
        if len(members) == 1:
            mean, std = 0.0, 1.0
        else:
            mean = s.mean()
            std = np.sqrt(((s - mean) ** 2).sum() / (len(s) - 1))
        out[members] = (s - mean) / (std + epsilon) if norm_adv_by_std_in_grpo else s - mean
    adv = out[:, None] * np.asarray(response_mask, f64)
    return adv, adv


def rloo_outcome_advantage(token_level_rewards, response_mask, index):
    """core_algos.py:444-493: n > 1 -> s * n / (n - 1) - mean * n / (n - 1); a single sample keeps s."""
    scores = np.asarray(token_level_rewards, np.float32).astype(f64).sum(-1)
    groups: dict = {}
    for i, u in enumerate(index):
        groups.setdefault(u, []).append(i)
    out = scores.copy()
    for members in groups.values():
        n = len(members)
        if n > 1:
            s = scores[members]
            out[members] = s * n / (n - 1) - s.mean() * n / (n - 1)
    adv = out[:, None] * np.asarray(response_mask, f64)
    return adv, adv


def reinforce_pp_baseline_outcome_advantage(token_level_rewards, response_mask, index):
    """core_algos.py:392-441: s - group mean (0 for a single sample), broadcast x mask, masked_whiten, x mask."""
    scores = np.asarray(token_level_rewards, np.float32).astype(f64).sum(-1)
    groups: dict = {}
    for i, u in enumerate(index):
        groups.setdefault(u, []).append(i)
    out = scores.copy()
    for members in groups.values():
        if len(members) > 1:
            out[members] = scores[members] - scores[members].mean()
    m = np.asarray(response_mask, f64)
    adv = masked_whiten(out[:, None] * m, response_mask) * m
    return adv, adv


def _groups(index):
    groups: dict = {}
    for i, u in enumerate(index):
        groups.setdefault(u, []).append(i)
    return groups


def opo_outcome_advantage(token_level_rewards, response_mask, index):
    """core_algos.py:495-546: s - sum(len * s) / sum(len) over the uid group (baseline 0 for a single sample),
    len = response_mask row sum; broadcast x mask."""
    scores = np.asarray(token_level_rewards, np.float32).astype(f64).sum(-1)
    lens = np.asarray(response_mask, f64).sum(-1)
    out = scores.copy()
    for members in _groups(index).values():
        if len(members) > 1:
            out[members] = scores[members] - (lens[members] * scores[members]).sum() / lens[members].sum()
    adv = out[:, None] * np.asarray(response_mask, f64)
    return adv, adv


def gpg_outcome_advantage(token_level_rewards, response_mask, index, f_norm=1.0):
    """core_algos.py:624-684: alpha * (s - group mean) / f_norm, alpha = B / max(#nonzero scores, 1) (group mean 0
    for a single sample); broadcast x mask."""
    scores = np.asarray(token_level_rewards, np.float32).astype(f64).sum(-1)
    B = scores.shape[0]
    alpha = B / max(int(np.count_nonzero(scores.astype(np.float32))), 1)
    out = np.empty_like(scores)
    for members in _groups(index).values():
        mean = scores[members].mean() if len(members) > 1 else 0.0
        out[members] = alpha * (scores[members] - mean) / f_norm
    adv = out[:, None] * np.asarray(response_mask, f64)
    return adv, adv


def grpo_passk_outcome_advantage(token_level_rewards, response_mask, index, epsilon=1e-6, norm_adv_by_std_in_grpo=True):
    """core_algos.py:327-386: per uid group (>= 2 samples, else ValueError), the best sample gets r_max - r_2nd
    (divided by the unbiased std + epsilon when normalising), every other sample 0; broadcast x mask."""
    scores = np.asarray(token_level_rewards, np.float32).astype(f64).sum(-1)
    out = np.zeros_like(scores)
    for u, members in _groups(index).items():
        if len(members) < 2:
            raise ValueError(f"Pass@k requires at least 2 samples per group. Got {len(members)} for group {u}.")
        s = scores[members]
        order = np.argsort(-s, kind="stable")
        a = s[order[0]] - s[order[1]]
        if norm_adv_by_std_in_grpo:
            a = a / (np.sqrt(((s - s.mean()) ** 2).sum() / (len(s) - 1)) + epsilon)
        out[members[order[0]]] = a
    adv = out[:, None] * np.asarray(response_mask, f64)
    return adv, adv


def remax_advantage_return(token_level_rewards, reward_baselines, response_mask):
    """core_algos.py:588-621: returns = reverse cumsum of rewards * mask (float32, from the last token); advantages
    = returns - baseline x mask."""
    r = np.asarray(token_level_rewards, np.float32) * np.asarray(response_mask, np.float32)
    ret = np.flip(np.cumsum(np.flip(r, -1), -1, dtype=np.float32), -1)
    adv = ret - np.asarray(reward_baselines, np.float32)[:, None] * np.asarray(response_mask, np.float32)
    return adv.astype(f64), ret.astype(f64)


def reinforce_pp_advantage_return(token_level_rewards, response_mask, gamma):
    """core_algos.py:550-586 (float32 scan in the reference's order)."""
    r = np.asarray(token_level_rewards, np.float32)
    m = np.asarray(response_mask, np.float32)
    B, T = r.shape
    ret = np.zeros((B, T), np.float32)
    running = np.zeros(B, np.float32)
    for t in reversed(range(T)):
        running = r[:, t] + np.float32(gamma) * running
        ret[:, t] = running
        running = running * m[:, t]
    adv = masked_whiten(ret.astype(f64), response_mask) * m
    return adv, ret.astype(f64)


def group_ids(index):
    """uid strings -> dense int32 group ids in order of first appearance (the CSR the HIP kernel takes)."""
    ids, order = {}, []
    for u in index:
        if u not in ids:
            ids[u] = len(ids)
        order.append(ids[u])
    return np.asarray(order, np.int32), len(ids)


# ---------------------------------------------------------------------------------------------
# compute_gae_advantage_return — core_algos.py:208-256
# ---------------------------------------------------------------------------------------------
def gae_advantage_return(token_level_rewards, values, response_mask, gamma, lam, values_bf16=False):
    """values_bf16: the values are a bf16 tensor in the reference (critic output, dp_critic.py:192), so
    `gamma * nextvalues` is bf16 tensor arithmetic there (rounded to bf16; core_algos.py:244)."""
    r = np.asarray(token_level_rewards, f64)
    v = np.asarray(values, f64)
    m = np.asarray(response_mask, f64)
    B, T = r.shape
    nextvalues = np.zeros(B)
    lastgaelam = np.zeros(B)
    adv = np.zeros((B, T))
    for t in reversed(range(T)):
        gv = gamma * nextvalues
        if values_bf16:
            gv = bf16_round(gv)
        delta = r[:, t] + gv - v[:, t]
        lg = delta + gamma * lam * lastgaelam
        nextvalues = v[:, t] * m[:, t] + (1 - m[:, t]) * nextvalues
        lastgaelam = lg * m[:, t] + (1 - m[:, t]) * lastgaelam
        adv[:, t] = lastgaelam
    returns = adv + v
    return masked_whiten(adv, response_mask), returns


# ---------------------------------------------------------------------------------------------
# compute_value_loss — core_algos.py:1230-1269 (+ the analytic d/d vpreds of dp_critic.py:237-240)
# ---------------------------------------------------------------------------------------------
def bf16_round(x):
    """Round to the nearest bfloat16 (ties to even), returned as float64."""
    a = np.ascontiguousarray(np.asarray(x, np.float32))
    u = a.view(np.uint32).astype(np.uint64)
    u = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return (u.astype(np.uint32).view(np.float32)).astype(f64)


def value_loss(vpreds, values, returns, response_mask, cliprange_value, loss_agg_mode="token-mean",
               loss_scale_factor=1.0, value_bf16=False):
    """Returns (vf_loss, vf_clipfrac, vpred_mean, d (vf_loss * loss_scale_factor) / d vpreds).

    clip_by_value (torch_functional.py:136-142) = torch.max(torch.min(vpreds, values + c), values - c); with
    bf16 critic outputs the bounds `values -/+ c` are bf16 tensors (rounded). Squared errors in float32
    against float32 returns (type promotion), reductions as agg_loss / masked_mean."""
    f32 = np.float32
    v = np.asarray(vpreds, f32)
    old = np.asarray(values, f32)
    ret = np.asarray(returns, f32)
    # tensor -/+ python float: float32 arithmetic with the scalar rounded to float32 (torch opmath)
    hi = old + f32(cliprange_value)
    lo = old - f32(cliprange_value)
    if value_bf16:  # bf16 tensor -/+ python float: the scalar is rounded to bf16 too (as torch computes it here)
        cb = f32(bf16_round(f32(cliprange_value)))
        hi, lo = bf16_round(old + cb).astype(f32), bf16_round(old - cb).astype(f32)
    y = np.minimum(v, hi)
    gy = np.where(v < hi, 1.0, np.where(v == hi, 0.5, 0.0))
    vc = np.maximum(y, lo)
    gc = np.where(y > lo, 1.0, np.where(y == lo, 0.5, 0.0))
    e1, e2 = v - ret, vc - ret
    l1, l2 = (e1 * e1).astype(f64), (e2 * e2).astype(f64)
    w1, w2 = _max_grad(l1, l2)
    lmax = np.maximum(l1, l2)
    vf_loss = 0.5 * agg_loss(lmax, response_mask, loss_agg_mode)
    vf_clipfrac = masked_mean((l2 > l1).astype(f64), response_mask)
    vpred_mean = masked_mean(v.astype(f64), response_mask)
    if value_bf16:  # masked_mean over a bf16 tensor: the sum is a bf16 tensor, the quotient promotes to fp32
        m = np.asarray(response_mask, f64)  # against the fp32 (mask.sum() + 1e-8) (torch_functional.py:163-185)
        vpred_mean = f32(bf16_round((v.astype(f64) * m).sum())) / f32(m.sum() + 1e-8)
    dl = w1 * 2.0 * e1.astype(f64) + w2 * 2.0 * e2.astype(f64) * gy * gc
    dv = loss_scale_factor * 0.5 * agg_loss_grad(response_mask, loss_agg_mode) * dl
    return vf_loss, vf_clipfrac, vpred_mean, dv


# ---------------------------------------------------------------------------------------------
# log-prob / entropy over the vocabulary — torch_functional.py:116-160 (+ backward)
# ---------------------------------------------------------------------------------------------
def logprob_entropy(logits, labels, temperature=1.0):
    """Returns (logp[N], entropy[N], softmax[N,V]) computed in float64 from the given logits."""
    z = np.asarray(logits, np.float32).astype(f64) / temperature
    zmax = z.max(-1, keepdims=True)
    e = np.exp(z - zmax)
    s = e.sum(-1, keepdims=True)
    lse = (np.log(s) + zmax)[:, 0]
    p = e / s
    logp = z[np.arange(z.shape[0]), labels] - lse
    ent = lse - (p * z).sum(-1)
    return logp, ent, p


def logprob_entropy_backward(logits, labels, dlogp, dentropy, temperature=1.0):
    """d/d logits of sum(dlogp*logp + dentropy*entropy)  (experimental/torch_functional.py:40-72)."""
    logp, ent, p = logprob_entropy(logits, labels, temperature)
    z = np.asarray(logits, np.float32).astype(f64) / temperature
    lse = logp - z[np.arange(z.shape[0]), labels]  # = -lse
    logsm = z + lse[:, None]
    onehot = np.zeros_like(p)
    onehot[np.arange(p.shape[0]), labels] = 1.0
    g = np.asarray(dlogp, f64)[:, None] * (onehot - p)
    g = g - np.asarray(dentropy, f64)[:, None] * p * (logsm + ent[:, None])
    return g / temperature


def fused_linear_logprob_entropy(hidden, weight, labels, temperature=1.0):
    """FusedLinearForPPO forward (experimental/torch_functional.py:20-37)."""
    logits = np.asarray(hidden, f64) @ np.asarray(weight, f64).T
    logp, ent, _ = logprob_entropy(logits, labels, temperature)
    return logp, ent


def fused_linear_backward(hidden, weight, labels, dlogp, dentropy, temperature=1.0):
    """FusedLinearForPPO backward (experimental/torch_functional.py:40-72): (d_hidden, d_weight)."""
    h = np.asarray(hidden, f64)
    w = np.asarray(weight, f64)
    logits = h @ w.T
    dlogits = logprob_entropy_backward(logits, labels, dlogp, dentropy, temperature)
    return dlogits @ w, dlogits.T @ h


# ---------------------------------------------------------------------------------------------
# rollout bookkeeping — torch_functional.py:226-246, utils/model.py:219, hf_rollout.py:151-160
# ---------------------------------------------------------------------------------------------
def get_response_mask(response_id, eos_token):
    eos = np.atleast_1d(np.asarray(eos_token))
    is_eos = np.isin(np.asarray(response_id), eos).astype(np.int64)
    return ((np.cumsum(is_eos, axis=1) - is_eos) == 0).astype(np.int64)


def compute_position_id_with_mask(mask):
    return np.clip(np.cumsum(np.asarray(mask, np.int64), axis=-1) - 1, 0, None)


def response_position_ids(prompt_position_ids, response_length):
    pos = np.asarray(prompt_position_ids, np.int64)
    delta = np.arange(1, response_length + 1, dtype=np.int64)[None, :]
    return np.concatenate([pos, pos[:, -1:] + delta], axis=-1)


# ---------------------------------------------------------------------------------------------
# decode-step token selection (HF generate semantics used by HFRollout, hf_rollout.py:112-124)
# ---------------------------------------------------------------------------------------------
def greedy(logits):
    """argmax with first-index tie-break (torch.argmax semantics)."""
    return np.asarray(logits).argmax(-1).astype(np.int64)


def philox4(seed, offset, counter):
    """Philox4x32-10 block (key = seed; counter words (c0, c1) = counter, (c2, c3) = offset) -> 4 words."""
    M0, M1, W0, W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    c = [counter & 0xFFFFFFFF, (counter >> 32) & 0xFFFFFFFF, offset & 0xFFFFFFFF, (offset >> 32) & 0xFFFFFFFF]
    for _ in range(10):
        p0 = M0 * c[0]
        p1 = M1 * c[2]
        c = [((p1 >> 32) ^ c[1] ^ k0) & 0xFFFFFFFF, p1 & 0xFFFFFFFF, ((p0 >> 32) ^ c[3] ^ k1) & 0xFFFFFFFF,
             p0 & 0xFFFFFFFF]
        k0 = (k0 + W0) & 0xFFFFFFFF
        k1 = (k1 + W1) & 0xFFFFFFFF
    return c


def philox_blocks(seed, offset, row, c0):
    """Philox4x32-10 blocks (key = seed; counter (c0, row), offset words (c2, c3)) for an array of counter low
    words c0 -> (len(c0), 4) uint32 (vectorised philox4)."""
    M0, M1, W0, W1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57), 0x9E3779B9, 0xBB67AE85
    mask = np.uint64(0xFFFFFFFF)
    c0 = np.asarray(c0, np.uint64)
    nb = c0.shape[0]
    c1 = np.full(nb, row & 0xFFFFFFFF, np.uint64)
    c2 = np.full(nb, offset & 0xFFFFFFFF, np.uint64)
    c3 = np.full(nb, (offset >> 32) & 0xFFFFFFFF, np.uint64)
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        c0, c1, c2, c3 = ((p1 >> np.uint64(32)) ^ c1 ^ np.uint64(k0)) & mask, p1 & mask, \
            ((p0 >> np.uint64(32)) ^ c3 ^ np.uint64(k1)) & mask, p0 & mask
        k0 = (k0 + W0) & 0xFFFFFFFF
        k1 = (k1 + W1) & 0xFFFFFFFF
    return np.stack([c0, c1, c2, c3], 1).astype(np.uint32)


def philox_words(seed, offset, row, V):
    """Word (i & 3) of block (row << 32 | i >> 2) for i < V (vectorised over the blocks)."""
    return philox_blocks(seed, offset, row, np.arange((V + 3) // 4, dtype=np.uint64)).reshape(-1)[:V]


def _log_clock(w):
    """ln(E) for E = -ln(1 - v) ~ Exp(1), v = ((w >> 8) + 0.5) / 2^24 (float32 uniform, as the HIP sampler)."""
    v = ((w >> np.uint32(8)).astype(np.float32) + np.float32(0.5)) * np.float32(1.0 / 16777216.0)
    return np.log(-np.log1p(-v))


def race_keys(z, seed, offset, row):
    """z_i - log(E_i), E_i = -log(1 - v_i) ~ Exp(1), v_i = ((w_i >> 8) + 0.5) / 2^24 (float32 math, as the
    HIP sampler); the argmax is a softmax(z) draw (exponential race / Gumbel-max)."""
    w = philox_words(seed, offset, row, z.shape[0])
    return np.asarray(z, np.float32) - _log_clock(w).astype(np.float32)


SELECT_SLICE = 2048  # tokens per slice of the two-level race (csrc/vocab.hip kSlice)


def slice_race_keys(z, keep, seed, offset, row):
    """Level 1 of the two-level race: slice s (tokens [2048 s, 2048 (s + 1))) has key
    ln(sum_{kept i in s} exp z_i) - ln(E_s), E_s from word (s & 3) of Philox block (row << 32 | 2^31 | s >> 2);
    -inf for a slice without kept tokens. float64 masses (the kernel sums float32 in a fixed order)."""
    z = np.asarray(z, np.float64)
    V = z.shape[0]
    S = -(-V // SELECT_SLICE)
    zz = np.full(S * SELECT_SLICE, -np.inf)
    zz[:V] = np.where(keep, z, -np.inf)
    zz = zz.reshape(S, SELECT_SLICE)
    m = zz.max(1)
    fin = np.isfinite(m)
    lnmass = np.full(S, -np.inf)
    lnmass[fin] = m[fin] + np.log(np.exp(zz[fin] - m[fin, None]).sum(1))
    w = philox_blocks(seed, offset, row, (1 << 31) + np.arange((S + 3) // 4, dtype=np.uint64)).reshape(-1)[:S]
    return lnmass - _log_clock(w)


def sample_row(logits, temperature, top_k, top_p, seed, offset, row, return_keys=False):
    """Reference semantics of one sampling step: temperature -> top-k -> top-p -> categorical draw.

    The draw is the HIP sampler's two-level exponential race over the kept tokens (slice_race_keys picks the
    slice, race_keys the token inside it; same Philox stream), so HIP and oracle pick the same token. HF uses
    torch.multinomial, whose one-sample path is the flat race argmax p_i / E_i: the same distribution (the
    first-arriving clock of a slice is an Exp(slice mass) clock)."""
    z = np.asarray(logits, np.float32).astype(f64) / temperature
    V = z.shape[0]
    keep = np.ones(V, bool)
    if top_k and 0 < top_k < V:
        kth = np.sort(z)[-top_k]
        keep &= z >= kth
    zs = np.where(keep, z, -np.inf)
    p = np.exp(zs - zs.max())
    p /= p.sum()
    if top_p < 1.0:
        order = np.argsort(-p, kind="stable")
        cum = np.cumsum(p[order])
        # HF TopPLogitsWarper: drop tokens whose ascending cumulative mass <= 1 - top_p, i.e. whose
        # strictly-higher-ranked mass already reaches top_p (the top token is always kept)
        drop = cum - p[order] >= top_p
        drop[0] = False
        keep2 = np.ones(V, bool)
        keep2[order[drop]] = False
        p = np.where(keep2, p, 0.0)
        p /= p.sum()
    z32 = (np.asarray(logits, np.float32) / np.float32(temperature)).astype(np.float32)
    kept = p > 0
    skeys = slice_race_keys(z32, kept, seed, offset, row)
    s = int(np.argmax(skeys))
    keys = np.where(kept, race_keys(z32, seed, offset, row), -np.inf)
    lo, hi = s * SELECT_SLICE, min(V, (s + 1) * SELECT_SLICE)
    tok = lo + int(np.argmax(keys[lo:hi]))
    return (tok, skeys, keys) if return_keys else tok


# ------------------------------------------------------------------------------------ A15 clip + AdamW
def grad_norm(g):
    """torch.nn.utils.clip_grad_norm_'s total 2-norm (dp_actor.py:282-298), accumulated in float64."""
    g = np.asarray(g, np.float64)
    return np.float32(np.sqrt(np.sum(g * g)))


def adamw_step(p, g, m, v, *, lr, beta1, beta2, eps, weight_decay, step, max_grad_norm, grad_norm_value):
    """In place on float32 arrays: clip_grad_norm_ (coef = max_norm / (norm + 1e-6), clamped to 1; a
    non-finite norm skips the step, dp_actor.py:292-297) then torch.optim.AdamW (decoupled weight decay,
    lerp first moment, bias-corrected denominator; fsdp_workers.py:454-459), in the float32 operation order of
    csrc/optim.hip's adam_one."""
    f = np.float32
    if not np.isfinite(grad_norm_value):
        return
    coef = f(1.0)
    if max_grad_norm > 0:
        coef = min(f(f(max_grad_norm) / (f(grad_norm_value) + f(1e-6))), f(1.0))
    step_size = f(lr / (1.0 - beta1 ** step))
    bc2_sqrt = f(np.sqrt(1.0 - beta2 ** step))
    gg = (g * coef).astype(f)
    p *= f(1.0) - f(lr) * f(weight_decay)
    m += (f(1.0) - f(beta1)) * (gg - m)
    v *= f(beta2)
    v += (f(1.0) - f(beta2)) * (gg * gg)
    denom = np.sqrt(v) / bc2_sqrt + f(eps)
    p += (-step_size) * (m / denom)
