"""Parity of the HIP kernels (through the C-ABI) with the reference's golden vectors and the CPU oracle.

GPU-only (``-m gpu``). Tolerances are stated per check: fp32 loss scalars within 1e-5 relative (the
north-star bar is 1e-4), per-token gradients within 2e-5 relative, integer/index outputs bit-exact.
"""

import numpy as np
import pytest
import torch

import oracle
from dots.rl_amd import native

pytestmark = pytest.mark.gpu
DEV = "cuda"
OUT_KEYS = ["pg_loss", "pg_clipfrac", "ppo_kl", "pg_clipfrac_lower", "entropy_loss", "kl_loss", "loss"]


def T(x, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(x)).to(DEV)
    return t.to(dtype) if dtype is not None else t


def run_k1(ins, cfg, mask_dtype=None, want_dent=True, given_count=False):
    old, lp, adv, mask, ent, ref = ins
    m = T(mask) if mask_dtype is None else T(mask).to(mask_dtype)
    tc = m.to(torch.float64).sum().reshape(1) if given_count else None
    out, dlp, dent = native.ppo_loss_fwd_bwd(
        T(old), T(lp), T(adv), m, T(ent), T(ref),
        clip_ratio_low=cfg["clip_ratio_low"], clip_ratio_high=cfg["clip_ratio_high"], clip_ratio_c=cfg["clip_ratio_c"],
        entropy_coeff=cfg["entropy_coeff"], kl_loss_coef=cfg["kl_loss_coef"],
        kl_loss_type=cfg["kl_loss_type"] if cfg["use_kl_loss"] else None, loss_agg_mode=cfg["loss_agg_mode"],
        loss_scale_factor=cfg["loss_scale_factor"], want_dlogp=True, want_dentropy=want_dent, token_count=tc)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    res = dict(zip(OUT_KEYS, o[:7]))
    res["mask_count"] = o[7]
    res["dlogp"] = dlp.cpu().numpy()
    res["dentropy"] = dent.cpu().numpy() if dent is not None else None
    return res


def test_ppo_loss_matches_reference_golden(golden):
    z, meta = golden("ppo_loss.npz")
    for ci, cfg in enumerate(meta["cases"]):
        g = lambda k: z[f"c{ci}_{k}"]  # noqa: E731
        ins = [g(k) for k in ["old_log_prob", "log_prob", "advantages", "response_mask", "entropy", "ref_log_prob"]]
        res = run_k1(ins, cfg)
        amb = oracle.clip_boundary_tokens(ins[0], ins[1], ins[2], ins[3], cfg["clip_ratio_low"], cfg["clip_ratio_high"],
                                          cfg["clip_ratio_c"])
        count = max(int(ins[3].sum()), 1)
        for k in OUT_KEYS:
            if k == "entropy_loss" and cfg["entropy_coeff"] == 0:
                continue
            if k == "kl_loss" and not cfg["use_kl_loss"]:
                continue
            atol = 1e-6 + (amb / count if "clipfrac" in k else 0.0)
            np.testing.assert_allclose(res[k], g(f"out_{k}"), rtol=1e-5, atol=atol, err_msg=f"case {ci} {k} {cfg}")
        np.testing.assert_allclose(res["dlogp"], g("out_dlogp"), rtol=2e-5, atol=1e-10, err_msg=f"case {ci} dlogp")
        np.testing.assert_allclose(res["dentropy"], g("out_dentropy"), rtol=2e-5, atol=1e-12, err_msg=f"case {ci} dent")


def rand_inputs(rng, B, R, hole_rows=True):
    old = (-rng.random((B, R)) * 5).astype(np.float32)
    lp = (old + rng.standard_normal((B, R)) * 0.3).astype(np.float32)
    adv = rng.standard_normal((B, R)).astype(np.float32)
    mask = np.zeros((B, R), np.int64)
    lens = rng.integers(1, R + 1, B)
    for i in range(B):
        mask[i, : lens[i]] = 1
    if hole_rows and B > 2:
        mask[1, ::3] = 0  # multi-turn style holes
    ent = (rng.random((B, R)) * 4).astype(np.float32)
    ref = (lp + rng.standard_normal((B, R)) * 0.1).astype(np.float32)
    return [old, lp, adv, mask, ent, ref]


@pytest.mark.parametrize("mode", oracle.AGG_MODES)
@pytest.mark.parametrize("mask_dtype", [torch.int64, torch.int32, torch.uint8, torch.bool, torch.float32])
@pytest.mark.parametrize("shape", [(3, 7), (8, 256), (37, 513), (64, 1000)])
@pytest.mark.parametrize("given_count", [False, True])  # token-mean: count pass + loss pass, or one pass
def test_ppo_loss_matches_oracle(mode, mask_dtype, shape, given_count):
    if given_count and mode != "token-mean":
        pytest.skip("token_count applies to token-mean")
    rng = np.random.default_rng(hash((mode, str(mask_dtype), shape)) % (2**32))
    ins = rand_inputs(rng, *shape)
    cfg = dict(clip_ratio_low=0.2, clip_ratio_high=0.28, clip_ratio_c=3.0, entropy_coeff=0.01, kl_loss_coef=0.001,
               kl_loss_type="low_var_kl", use_kl_loss=True, loss_agg_mode=mode, loss_scale_factor=0.25)
    res = run_k1(ins, cfg, mask_dtype, given_count=given_count)
    ref = oracle.actor_loss(*ins, loss_agg_mode=mode, clip_ratio_low=0.2, clip_ratio_high=0.28, clip_ratio_c=3.0,
                            entropy_coeff=0.01, use_kl_loss=True, kl_loss_type="low_var_kl", kl_loss_coef=0.001,
                            loss_scale_factor=0.25)
    amb = oracle.clip_boundary_tokens(*ins[:4], 0.2, 0.28, 3.0)
    count = int(ins[3].sum())
    for k in OUT_KEYS:
        atol = 1e-6 + (amb / count if "clipfrac" in k else 0.0)
        np.testing.assert_allclose(res[k], ref[k], rtol=1e-5, atol=atol, err_msg=k)
    assert res["mask_count"] == count
    np.testing.assert_allclose(res["dlogp"], ref["dlogp"], rtol=2e-5, atol=1e-11)
    np.testing.assert_allclose(res["dentropy"], ref["dentropy"], rtol=2e-5, atol=1e-12)


def test_ppo_loss_forward_only_and_no_optional_inputs():
    rng = np.random.default_rng(0)
    old, lp, adv, mask, ent, ref = rand_inputs(rng, 16, 200)
    out, dlp, dent = native.ppo_loss_fwd_bwd(T(old), T(lp), T(adv), T(mask), want_dlogp=False)
    assert dlp is None and dent is None
    r = oracle.policy_loss_vanilla(old, lp, adv, mask)
    o = out.cpu().numpy()
    np.testing.assert_allclose(o[:4], np.array(r[:4], np.float64), rtol=1e-5, atol=1e-6)


def test_ppo_loss_deterministic_and_large():
    """2^22 tokens: bitwise run-to-run reproducibility + agreement with a plain torch fp32 reference."""
    B, R = 4096, 1024
    g = torch.Generator(device=DEV).manual_seed(1)
    old = -torch.rand(B, R, device=DEV, generator=g) * 5
    lp = old + torch.randn(B, R, device=DEV, generator=g) * 0.3
    adv = torch.randn(B, R, device=DEV, generator=g)
    mask = (torch.rand(B, R, device=DEV, generator=g) > 0.1).to(torch.int64)
    ent = torch.rand(B, R, device=DEV, generator=g)
    ref = lp + torch.randn(B, R, device=DEV, generator=g) * 0.1
    kw = dict(clip_ratio_low=0.2, clip_ratio_high=0.2, clip_ratio_c=3.0, entropy_coeff=0.001, kl_loss_coef=0.001,
              kl_loss_type="low_var_kl", loss_agg_mode="token-mean", loss_scale_factor=1.0, want_dentropy=True)
    o1, d1, e1 = native.ppo_loss_fwd_bwd(old, lp, adv, mask, ent, ref, **kw)
    o1, d1, e1 = o1.clone(), d1.clone(), e1.clone()
    o2, d2, e2 = native.ppo_loss_fwd_bwd(old, lp, adv, mask, ent, ref, **kw)
    assert torch.equal(o1, o2) and torch.equal(d1, d2) and torch.equal(e1, e2)
    # one-pass form with the caller's token count: the same bits
    tc = mask.to(torch.float64).sum().reshape(1)
    o3, d3, e3 = native.ppo_loss_fwd_bwd(old, lp, adv, mask, ent, ref, token_count=tc, **kw)
    assert torch.equal(o1, o3) and torch.equal(d1, d3) and torch.equal(e1, e3)
    # plain torch fp32 reference (same formulas as core_algos.py:815-889 / dp_actor.py:419-466)
    x = lp.clone().requires_grad_(True)
    e = ent.clone().requires_grad_(True)
    nkl = torch.clamp(x - old, -20, 20)
    ratio = torch.exp(nkl)
    l1, l2 = -adv * ratio, -adv * torch.clamp(ratio, 0.8, 1.2)
    c1 = torch.maximum(l1, l2)
    l3 = -adv * 3.0
    pg = torch.where(adv < 0, torch.min(l3, c1), c1)
    mf = mask.float()
    mm = lambda v: (torch.where(mask.bool(), v, 0.0) * mf).sum() / (mf.sum() + 1e-8)  # noqa: E731
    kl = torch.clamp(ref - x, -20, 20)
    kld = torch.clamp(torch.exp(kl) - kl - 1, -10, 10)
    loss = mm(pg) - mm(e) * 0.001 + mm(kld) * 0.001
    loss.backward()
    torch.testing.assert_close(o1[6], loss.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(d1, x.grad, rtol=1e-4, atol=1e-12)
    torch.testing.assert_close(e1, e.grad, rtol=1e-5, atol=1e-14)


def test_kl_penalty_and_agg_loss():
    rng = np.random.default_rng(3)
    lp = rng.standard_normal(5000).astype(np.float32)
    ref = (lp + rng.standard_normal(5000) * 5).astype(np.float32)
    for kl in ["kl", "abs", "mse", "low_var_kl"]:
        got = native.kl_penalty(T(lp), T(ref), kl).cpu().numpy()
        np.testing.assert_allclose(got, oracle.kl_penalty(lp, ref, kl)[0], rtol=2e-6, atol=2e-6, err_msg=kl)
    x = rng.standard_normal((33, 77)).astype(np.float32)
    m = (rng.random((33, 77)) > 0.4).astype(np.int64)
    m[:, 0] = 1
    for mode in oracle.AGG_MODES:
        got = native.agg_loss(T(x), T(m), mode).item()
        np.testing.assert_allclose(got, oracle.agg_loss(x, m, mode), rtol=1e-5, atol=1e-7, err_msg=mode)


# ---------------------------------------------------------------------------------------------------- K2
def regen_logits(case):
    rng = np.random.default_rng(case["seed"])
    x = (rng.standard_normal((case["N"], case["V"]), dtype=np.float32) * np.float32(case["scale"])).astype(np.float32)
    labels = rng.integers(0, case["V"], size=(case["N"],), dtype=np.int64)
    dlogp = rng.standard_normal((case["N"],), dtype=np.float32)
    dent = rng.standard_normal((case["N"],), dtype=np.float32)
    return x, labels, dlogp, dent


@pytest.mark.parametrize("ci", [0, 1, 2, 3])
@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_logprob_entropy_matches_reference_golden(golden, ci, dt):
    z, meta = golden("logprob.npz")
    case = meta["cases"][ci]
    x, labels, dlogp, dent = regen_logits(case)
    logits = T(x) if dt == "fp32" else T(x).to(torch.bfloat16)
    lp, ent, lse = native.logprob_entropy_fwd(logits, T(labels))
    np.testing.assert_allclose(lp.cpu().numpy(), z[f"c{ci}_{dt}_logp"], rtol=1e-5, atol=3e-5)
    np.testing.assert_allclose(ent.cpu().numpy(), z[f"c{ci}_{dt}_entropy"], rtol=6e-5, atol=3e-5)
    g_lp = native.logprob_entropy_bwd(logits, T(labels), 1.0, T(dlogp), None, lse, ent, out_dtype=torch.float32)
    g_en = native.logprob_entropy_bwd(logits, T(labels), 1.0, None, T(dent), lse, ent, out_dtype=torch.float32)
    g_lp, g_en = g_lp.cpu().numpy(), g_en.cpu().numpy()
    if case["inputs_from_seed"]:
        idx = np.arange(0, x.size, 997)
        np.testing.assert_allclose(g_lp.reshape(-1)[idx], z[f"c{ci}_{dt}_dlogits_lp_sample"], rtol=1e-4, atol=1e-9)
        np.testing.assert_allclose(g_en.reshape(-1)[idx], z[f"c{ci}_{dt}_dlogits_ent_sample"], rtol=2e-3, atol=1e-9)
    else:
        np.testing.assert_allclose(g_lp, z[f"c{ci}_{dt}_dlogits_lp"], rtol=1e-4, atol=1e-8)
        np.testing.assert_allclose(g_en, z[f"c{ci}_{dt}_dlogits_ent"], rtol=2e-3, atol=1e-7)


def test_logprob_temperature_and_strided_rows():
    rng = np.random.default_rng(9)
    x = (rng.standard_normal((12, 1003)) * 4).astype(np.float32)
    labels = rng.integers(0, 1003, 12)
    full = T(np.concatenate([x, np.zeros((12, 5), np.float32)], 1))[:, :1003]  # ld = 1008, V = 1003
    for temp in (1.0, 0.7, 1.5):
        lp, ent, _ = native.logprob_entropy_fwd(full, T(labels), temperature=temp)
        rlp, rent, _ = oracle.logprob_entropy(x / np.float32(temp), labels)
        np.testing.assert_allclose(lp.cpu().numpy(), rlp, rtol=1e-5, atol=2e-5)
        np.testing.assert_allclose(ent.cpu().numpy(), rent, rtol=1e-5, atol=2e-5)


def test_logprob_bf16_inplace_backward():
    rng = np.random.default_rng(10)
    x = (rng.standard_normal((6, 4096)) * 3).astype(np.float32)
    labels = rng.integers(0, 4096, 6)
    logits = T(x).to(torch.bfloat16)
    xb = logits.float().cpu().numpy()
    lp, ent, lse = native.logprob_entropy_fwd(logits, T(labels))
    dl = rng.standard_normal(6).astype(np.float32)
    de = rng.standard_normal(6).astype(np.float32)
    native.logprob_entropy_bwd(logits, T(labels), 1.0, T(dl), T(de), lse, ent, out=logits)  # in place
    ref = oracle.logprob_entropy_backward(xb, labels, dl, de)
    np.testing.assert_allclose(logits.float().cpu().numpy(), ref, rtol=1e-2, atol=1e-4)


# ---------------------------------------------------------------------------------------------------- K3/K5
def csr(uid):
    ids, G = oracle.group_ids(list(uid))
    order = np.argsort(ids, kind="stable").astype(np.int32)
    offsets = np.zeros(G + 1, np.int32)
    np.add.at(offsets, ids + 1, 1)
    return ids, np.cumsum(offsets).astype(np.int32), order, G


def test_grpo_matches_reference_golden(golden):
    z, meta = golden("grpo.npz")
    for ci, cfg in enumerate(meta["cases"]):
        ids, off, mem, G = csr(z[f"c{ci}_uid"])
        adv, ret = native.grpo_outcome_advantage(T(z[f"c{ci}_rewards"]), T(z[f"c{ci}_mask"]), T(ids), T(off), T(mem), G,
                                                 cfg["epsilon"], cfg["norm_adv_by_std_in_grpo"])
        np.testing.assert_allclose(adv.cpu().numpy(), z[f"c{ci}_adv"], rtol=1e-5, atol=1e-6, err_msg=str(cfg))
        np.testing.assert_allclose(ret.cpu().numpy(), z[f"c{ci}_ret"], rtol=1e-5, atol=1e-6)


def test_rloo_and_reinforce_pp_baseline_match_reference_golden(golden):
    from dots.rl_amd import core_algos

    z, meta = golden("group_adv.npz")
    fns = {"rloo": core_algos.compute_rloo_outcome_advantage,
           "reinforce_plus_plus_baseline": core_algos.compute_reinforce_plus_plus_baseline_outcome_advantage}
    assert core_algos.get_adv_estimator_fn("rloo") is fns["rloo"]
    for ci, c in enumerate(meta["cases"]):
        adv, ret = fns[c["estimator"]](T(z[f"c{ci}_rewards"]), T(z[f"c{ci}_mask"]), list(z[f"c{ci}_uid"]))
        np.testing.assert_allclose(adv.cpu().numpy(), z[f"c{ci}_adv"], rtol=2e-5, atol=2e-6, err_msg=str(c))
        np.testing.assert_allclose(ret.cpu().numpy(), z[f"c{ci}_ret"], rtol=2e-5, atol=2e-6, err_msg=str(c))


def test_opo_gpg_passk_remax_match_reference_golden(golden):
    """K3 OPO / GPG / pass@k modes and the ReMax scan, through the registry the trainer uses, against the
    reference estimators (more_adv.npz); pass@k refuses a singleton group with the reference's message."""
    from dots.rl_amd import core_algos
    from dots.rl_amd.config import to_attr

    z, meta = golden("more_adv.npz")
    for ci, c in enumerate(meta["cases"]):
        est = c["estimator"]
        r, m = T(z[f"c{ci}_rewards"]), T(z[f"c{ci}_mask"])
        if est == "remax":
            fn = core_algos.get_adv_estimator_fn("remax")
            adv, ret = fn(token_level_rewards=r, reward_baselines=T(z[f"c{ci}_baselines"]), response_mask=m,
                          config=None)
        else:
            name = "grpo_passk" if est.startswith("grpo_passk") else est
            fn = core_algos.get_adv_estimator_fn(name)
            cfg = to_attr({"norm_adv_by_std_in_grpo": est.endswith("_std")})
            adv, ret = fn(token_level_rewards=r, response_mask=m, index=list(z[f"c{ci}_uid"]), config=cfg)
        np.testing.assert_allclose(adv.cpu().numpy(), z[f"c{ci}_adv"], rtol=2e-5, atol=2e-6, err_msg=str(c))
        np.testing.assert_allclose(ret.cpu().numpy(), z[f"c{ci}_ret"], rtol=2e-5, atol=2e-6, err_msg=str(c))
    with pytest.raises(ValueError) as e:
        core_algos.get_adv_estimator_fn("grpo_passk")(
            token_level_rewards=torch.ones(3, 4, device=DEV), response_mask=torch.ones(3, 4, device=DEV),
            index=["a", "a", "b"], config=to_attr({"norm_adv_by_std_in_grpo": True}))
    assert str(e.value) == meta["passk_singleton_error"]


def test_reinforce_pp_matches_reference_golden(golden):
    from dots.rl_amd import core_algos
    from dots.rl_amd.config import to_attr

    z, meta = golden("rfpp.npz")
    fn = core_algos.get_adv_estimator_fn("reinforce_plus_plus")
    for ci, c in enumerate(meta["cases"]):
        adv, ret = fn(token_level_rewards=T(z[f"c{ci}_rewards"]), response_mask=T(z[f"c{ci}_mask"]),
                      config=to_attr({"gamma": c["gamma"]}))
        np.testing.assert_allclose(adv.cpu().numpy(), z[f"c{ci}_adv"], rtol=2e-5, atol=2e-6)
        np.testing.assert_allclose(ret.cpu().numpy(), z[f"c{ci}_ret"], rtol=1e-6, atol=1e-7)


def test_gpg_actor_loss_matches_reference_golden(golden):
    """K1 in GPG mode (policy_loss.loss_mode=gpg) vs the reference's compute_policy_loss_gpg composed into the
    dp_actor total loss (entropy bonus, KL, loss scale) and its autograd gradients."""
    z, meta = golden("gpg_loss.npz")
    for ci, c in enumerate(meta["cases"]):
        g = lambda k: T(z[f"c{ci}_{k}"])  # noqa: E731
        out, dlp, dent = native.ppo_loss_fwd_bwd(
            g("old_log_prob"), g("log_prob"), g("advantages"), g("response_mask"), g("entropy"), g("ref_log_prob"),
            entropy_coeff=c["entropy_coeff"], kl_loss_coef=c["kl_loss_coef"], kl_loss_type=c["kl_loss_type"],
            loss_agg_mode=c["loss_agg_mode"], loss_scale_factor=c["loss_scale_factor"], want_dentropy=True,
            policy_loss="gpg")
        o = out.cpu().numpy()
        np.testing.assert_allclose(o[0], z[f"c{ci}_out_pg_loss"], rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(o[6], z[f"c{ci}_out_loss"], rtol=1e-5, atol=1e-7)
        assert o[1] == 0 and o[2] == 0 and o[3] == 0
        np.testing.assert_allclose(dlp.cpu().numpy(), z[f"c{ci}_out_dlogp"], rtol=2e-5, atol=1e-9)
        np.testing.assert_allclose(dent.cpu().numpy(), z[f"c{ci}_out_dentropy"], rtol=2e-5, atol=1e-9)


def test_gspo_geo_mean_actor_loss_matches_reference_golden(golden):
    """The sequence-level losses (policy_loss.loss_mode gspo / geo_mean) through the K1 entry point vs the reference's
    losses composed into the dp_actor total loss and its autograd gradients (seq_loss.npz): sequence ratios past
    GSPO's clamp at 10, zero advantages, clip edges, every aggregation mode for the entropy / KL terms."""
    z, meta = golden("seq_loss.npz")
    for ci, c in enumerate(meta["cases"]):
        g = lambda k: T(z[f"c{ci}_{k}"])  # noqa: E731
        out, dlp, dent = native.ppo_loss_fwd_bwd(
            g("old_log_prob"), g("log_prob"), g("advantages"), g("response_mask"), g("entropy"), g("ref_log_prob"),
            clip_ratio_low=c["clip_ratio_low"], clip_ratio_high=c["clip_ratio_high"],
            entropy_coeff=c["entropy_coeff"], kl_loss_coef=c["kl_loss_coef"], kl_loss_type=c["kl_loss_type"],
            loss_agg_mode=c["loss_agg_mode"], loss_scale_factor=c["loss_scale_factor"], want_dentropy=True,
            policy_loss=c["policy_loss"])
        o = out.cpu().numpy()
        np.testing.assert_allclose(o[0], z[f"c{ci}_out_pg_loss"], rtol=2e-5, atol=1e-6, err_msg=str(c))
        np.testing.assert_allclose(o[6], z[f"c{ci}_out_loss"], rtol=2e-5, atol=1e-6, err_msg=str(c))
        np.testing.assert_allclose(o[[1, 2, 3]], z[f"c{ci}_out_clip"], rtol=2e-5, atol=1e-6, err_msg=str(c))
        np.testing.assert_allclose(o[4], z[f"c{ci}_out_entropy_loss"], rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(o[5], z[f"c{ci}_out_kl_loss"], rtol=1e-5, atol=1e-7)
        d = z[f"c{ci}_out_dlogp"]
        np.testing.assert_allclose(dlp.cpu().numpy(), d, rtol=2e-4, atol=1e-6 * np.abs(d).max(), err_msg=str(c))
        np.testing.assert_allclose(dent.cpu().numpy(), z[f"c{ci}_out_dentropy"], rtol=2e-5, atol=1e-9)


@pytest.mark.parametrize("policy", ["gspo", "geo_mean"])
@pytest.mark.parametrize("mode", ["token-mean", "seq-mean-token-mean"])
def test_seq_policy_loss_at_size_matches_oracle(policy, mode):
    """GSPO / GMPO at a micro-batch shape (64 x 1024, ragged rows) vs the oracle; deterministic run to run."""
    rng = np.random.default_rng(17)
    B, R = 64, 1024
    old = (-rng.random((B, R)) * 5).astype(np.float32)
    lp = (old + rng.standard_normal((B, R)) * 0.05 + rng.standard_normal((B, 1)) * 0.1).astype(np.float32)
    adv = np.repeat(rng.standard_normal((B, 1)), R, 1).astype(np.float32)
    mask = (np.arange(R)[None, :] < rng.integers(1, R + 1, (B, 1))).astype(np.int64)
    ent = rng.random((B, R)).astype(np.float32)
    ref = (lp + rng.standard_normal((B, R)) * 0.1).astype(np.float32)
    kw = dict(clip_ratio_low=0.2, clip_ratio_high=0.28, entropy_coeff=0.001, kl_loss_coef=0.001,
              kl_loss_type="low_var_kl", loss_agg_mode=mode, loss_scale_factor=0.5, want_dentropy=True,
              policy_loss=policy)
    out, dlp, dent = native.ppo_loss_fwd_bwd(T(old), T(lp), T(adv), T(mask), T(ent), T(ref), **kw)
    want = oracle.actor_loss(old, lp, adv, mask, ent, ref, loss_agg_mode=mode, clip_ratio_low=0.2,
                             clip_ratio_high=0.28, clip_ratio_c=3.0, entropy_coeff=0.001, use_kl_loss=True,
                             kl_loss_type="low_var_kl", kl_loss_coef=0.001, loss_scale_factor=0.5, policy_loss=policy)
    o = out.cpu().numpy()
    np.testing.assert_allclose(o[0], want["pg_loss"], rtol=2e-5, atol=1e-7)
    np.testing.assert_allclose(o[6], want["loss"], rtol=2e-5, atol=1e-7)
    np.testing.assert_allclose(o[[1, 2, 3]], [want["pg_clipfrac"], want["ppo_kl"], want["pg_clipfrac_lower"]],
                               rtol=1e-4, atol=1e-6)
    d = want["dlogp"]
    np.testing.assert_allclose(dlp.cpu().numpy(), d, rtol=2e-4, atol=1e-6 * np.abs(d).max())
    np.testing.assert_allclose(dent.cpu().numpy(), want["dentropy"], rtol=2e-5, atol=1e-12)
    out2, dlp2, _ = native.ppo_loss_fwd_bwd(T(old), T(lp), T(adv), T(mask), T(ent), T(ref), **kw)
    assert torch.equal(out, out2) and torch.equal(dlp, dlp2)


def test_cov_actor_loss_matches_reference_golden(golden):
    """Clip-Cov / KL-Cov through the K1 entry point vs the reference losses composed into the dp_actor total loss
    (cov_loss.npz; clip_cov where every candidate is taken, so the reference's torch.randperm draw is moot)."""
    z, meta = golden("cov_loss.npz")
    for ci, c in enumerate(meta["cases"]):
        g = lambda k: T(z[f"c{ci}_{k}"])  # noqa: E731
        out, dlp, dent = native.ppo_loss_fwd_bwd(
            g("old_log_prob"), g("log_prob"), g("advantages"), g("response_mask"), g("entropy"), g("ref_log_prob"),
            clip_ratio_low=c["clip_ratio_low"], clip_ratio_high=c["clip_ratio_high"],
            entropy_coeff=c["entropy_coeff"], kl_loss_coef=c["kl_loss_coef"], kl_loss_type=c["kl_loss_type"],
            loss_agg_mode=c["loss_agg_mode"], loss_scale_factor=c["loss_scale_factor"], want_dentropy=True,
            policy_loss=c["policy_loss"], cov_ratio=c["cov_ratio"], clip_cov_lb=c["clip_cov_lb"],
            clip_cov_ub=c["clip_cov_ub"], ppo_kl_coef=c["ppo_kl_coef"], cov_seed=123)
        o = out.cpu().numpy()
        np.testing.assert_allclose(o[0], z[f"c{ci}_out_pg_loss"], rtol=2e-5, atol=1e-6, err_msg=str(c))
        np.testing.assert_allclose(o[6], z[f"c{ci}_out_loss"], rtol=2e-5, atol=1e-6, err_msg=str(c))
        np.testing.assert_allclose(o[[1, 2, 3]], z[f"c{ci}_out_clip"], rtol=2e-5, atol=1e-6, err_msg=str(c))
        d = z[f"c{ci}_out_dlogp"]
        np.testing.assert_allclose(dlp.cpu().numpy(), d, rtol=2e-4, atol=1e-6 * np.abs(d).max(), err_msg=str(c))
        np.testing.assert_allclose(dent.cpu().numpy(), z[f"c{ci}_out_dentropy"], rtol=2e-5, atol=1e-9)


@pytest.mark.parametrize("policy,ratio", [("kl_cov", 0.0002), ("kl_cov", 0.01), ("clip_cov", 0.0002), ("clip_cov", 0.002)])
def test_cov_policy_loss_at_size_matches_oracle(policy, ratio):
    """Clip-Cov / KL-Cov at 64 x 1024 (ragged rows) vs the oracle: the same top-k tokens (kl_cov) and the same
    seeded random subset of the candidates (clip_cov, many more candidates than clip_num); deterministic; a new
    seed draws another clip_cov subset of the same size."""
    rng = np.random.default_rng(23)
    B, R = 64, 1024
    old = (-rng.random((B, R)) * 5).astype(np.float32)
    lp = (old + rng.standard_normal((B, R)) * 0.3).astype(np.float32)
    adv = (rng.standard_normal((B, R)) * 2).astype(np.float32)
    mask = (np.arange(R)[None, :] < rng.integers(1, R + 1, (B, 1))).astype(np.int64)
    kw = dict(clip_ratio_low=0.2, clip_ratio_high=0.28, loss_agg_mode="token-mean", loss_scale_factor=1.0,
              policy_loss=policy, cov_ratio=ratio, clip_cov_lb=1.0, clip_cov_ub=5.0, ppo_kl_coef=0.1, cov_seed=77)
    out, dlp, _ = native.ppo_loss_fwd_bwd(T(old), T(lp), T(adv), T(mask), **kw)
    want = oracle.actor_loss(old, lp, adv, mask, np.zeros_like(old), lp, loss_agg_mode="token-mean",
                             clip_ratio_low=0.2, clip_ratio_high=0.28, clip_ratio_c=3.0, entropy_coeff=0.0,
                             use_kl_loss=False, kl_loss_type="kl", kl_loss_coef=0.0, loss_scale_factor=1.0,
                             policy_loss=policy, cov_ratio=ratio, clip_cov_lb=1.0, clip_cov_ub=5.0, ppo_kl_coef=0.1,
                             cov_seed=77)
    o = out.cpu().numpy()
    np.testing.assert_allclose(o[0], want["pg_loss"], rtol=2e-5, atol=1e-7)
    np.testing.assert_allclose(o[[1, 2, 3]], [want["pg_clipfrac"], want["ppo_kl"], want["pg_clipfrac_lower"]],
                               rtol=1e-4, atol=1e-7)
    d = want["dlogp"]
    np.testing.assert_allclose(dlp.cpu().numpy(), d, rtol=2e-4, atol=1e-6 * np.abs(d).max())
    out2, dlp2, _ = native.ppo_loss_fwd_bwd(T(old), T(lp), T(adv), T(mask), **kw)
    assert torch.equal(out, out2) and torch.equal(dlp, dlp2)
    if policy == "clip_cov":
        _, _, _, _, _, sel = oracle.policy_loss_clip_cov(old, lp, adv, mask, "token-mean", 0.2, 0.28, ratio, 1.0, 5.0,
                                                         77, return_selected=True)
        assert sel.sum() == max(int(ratio * mask.sum()), 1)
        kw["cov_seed"] = 78
        out3, _, _ = native.ppo_loss_fwd_bwd(T(old), T(lp), T(adv), T(mask), **kw)
        assert out3[1].item() == out[1].item()  # same subset size (pg_clipfrac), another draw
        assert out3[0].item() != out[0].item()


def test_gae_matches_reference_golden(golden):
    z, meta = golden("gae.npz")
    for ci, cfg in enumerate(meta["cases"]):
        adv, ret = native.gae_advantage_return(T(z[f"c{ci}_rewards"]), T(z[f"c{ci}_values"]), T(z[f"c{ci}_mask"]),
                                               cfg["gamma"], cfg["lam"])
        np.testing.assert_allclose(adv.cpu().numpy(), z[f"c{ci}_adv"], rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(ret.cpu().numpy(), z[f"c{ci}_ret"], rtol=1e-5, atol=1e-5)


# ---------------------------------------------------------------------------------------------------- A4/A5
def test_masks_and_positions_match_reference_golden(golden):
    z, _ = golden("masks.npz")
    for key, eos in [("doc_mask_eos1", [1]), ("doc_mask_eos12", [1, 2])]:
        got = native.response_mask(T(z["doc_responses"]), T(np.array(eos, np.int64))).cpu().numpy()
        np.testing.assert_array_equal(got, z[key])
    for key, eos in [("rand_mask_eos7", [7]), ("rand_mask_eos7_9_11", [7, 9, 11])]:
        got = native.response_mask(T(z["rand_responses"]), T(np.array(eos, np.int64))).cpu().numpy()
        np.testing.assert_array_equal(got, z[key])
    pos = native.position_ids(T(z["prompt_attention_mask"])).cpu().numpy()
    np.testing.assert_array_equal(pos, z["prompt_position_ids"])
    P = pos.shape[1]
    full = torch.zeros(z["full_position_ids"].shape, dtype=torch.int64, device=DEV)
    full[:, :P] = T(pos)
    native.response_position_ids_(full, P)
    np.testing.assert_array_equal(full.cpu().numpy(), z["full_position_ids"])


# ---------------------------------------------------------------------------------------------------- K4
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_greedy_bit_exact_with_ties_and_nan(dt):
    g = torch.Generator(device=DEV).manual_seed(4)
    logits = (torch.randn(64, 151936, device=DEV, generator=g) * 3).to(dt)
    logits[3, 100] = logits[3, 7] = 1e4  # tie -> first index
    logits[5, 999] = float("nan")  # NaN is the argmax (torch.argmax)
    logits[6, :] = -float("inf")
    out = torch.full((64,), -1, dtype=torch.int64, device=DEV)
    native.select_tokens(logits, out)
    assert torch.equal(out, torch.argmax(logits, dim=-1))
    assert out[3].item() == 7 and out[5].item() == 999


def test_greedy_writes_strided_column_and_handles_eos():
    V = 50
    logits = torch.zeros(4, V, device=DEV)
    logits[torch.arange(4), torch.tensor([3, 9, 9, 5])] = 5.0
    responses = torch.full((4, 10), -7, dtype=torch.int64, device=DEV)
    unfinished = torch.tensor([1, 1, 0, 1], dtype=torch.int32, device=DEV)
    eos = torch.tensor([9, 5], dtype=torch.int64, device=DEV)
    native.select_tokens(logits, responses[:, 2], pad_token_id=0, eos_ids=eos, unfinished=unfinished)
    assert responses[:, 2].tolist() == [3, 9, 0, 5]
    assert unfinished.tolist() == [1, 0, 0, 0]
    assert (responses[:, [0, 1, 3]] == -7).all()


@pytest.mark.parametrize("dt,V", [(torch.float32, 151936), (torch.bfloat16, 151936), (torch.bfloat16, 1001),
                                  (torch.float32, 77), (torch.bfloat16, 4096), (torch.float32, 6145)])
def test_sampling_matches_oracle_race(dt, V):
    """Sampled tokens == the oracle's two-level exponential race on the same Philox stream (slice race on the
    slice masses, then the token race inside the winning slice). A row whose two best oracle slice keys (float64
    masses vs the kernel's float32 sums) or two best token keys are within float32 rounding may pick either."""
    rng = np.random.default_rng(12)
    N = 48
    x = (rng.standard_normal((N, V)) * 2).astype(np.float32)
    logits = T(x).to(dt)
    xs = logits.float().cpu().numpy()
    out = torch.empty(N, dtype=torch.int64, device=DEV)
    seed, step, temp = 1234, 17, 0.8
    native.select_tokens(logits, out, do_sample=True, temperature=temp, seed=seed, step=step, row_base=100)
    got = out.cpu().numpy()
    exact = 0
    for i in range(N):
        want, skeys, keys = oracle.sample_row(xs[i], temp, 0, 1.0, seed, step, 100 + i, return_keys=True)
        if got[i] == want:
            exact += 1
            continue
        sg, sw = got[i] // oracle.SELECT_SLICE, want // oracle.SELECT_SLICE
        if sg != sw:
            assert abs(skeys[sg] - skeys[sw]) <= 1e-5 * max(1.0, abs(skeys[sw])), (i, got[i], want)
        else:
            assert abs(keys[got[i]] - keys[want]) <= 1e-5 * max(1.0, abs(keys[want])), (i, got[i], want)
    assert exact >= N - 2, exact


def test_sampling_distribution_across_slices():
    """Two-level race draw frequencies: 8192 rows of the same 3-slice row (V = 5000) whose mass sits in a few
    tokens spread over the slices and a flat background; temperature 0.7; distinct Philox counters per row."""
    V, N = 5000, 8192
    z = torch.full((V,), -4.0)
    hot = [7, 2047, 2048, 3000, 4999]
    z[hot] = torch.tensor([1.0, 0.2, 0.6, -0.5, 1.3])
    out = torch.empty(N, dtype=torch.int64, device=DEV)
    native.select_tokens(z.repeat(N, 1).to(DEV), out, do_sample=True, temperature=0.7, seed=3, step=2)
    got = out.cpu().numpy()
    p = torch.softmax(z / 0.7, 0).numpy().astype(np.float64)
    bins = np.array(hot + [-1])  # the hot tokens, then everything else
    freq = np.array([(got == h).mean() for h in hot] + [(~np.isin(got, hot)).mean()])
    q = np.append(p[hot], 1.0 - p[hot].sum())
    assert np.abs(freq - q).max() < 4 * np.sqrt(q.max() * (1 - q.max()) / N), (bins, freq, q)
    # slice frequencies
    fs = np.bincount(got // 2048, minlength=3) / N
    qs = np.array([p[:2048].sum(), p[2048:4096].sum(), p[4096:].sum()])
    assert np.abs(fs - qs).max() < 4 * np.sqrt(0.25 / N), (fs, qs)


def _hf_kept(z, top_k, top_p):
    """Kept set of HF TopKLogitsWarper -> TopPLogitsWarper on fp32 scores z (oracle.sample_row's rule)."""
    V = z.shape[0]
    keep = np.ones(V, bool)
    if 0 < top_k < V:
        keep &= z >= np.sort(z)[-top_k]
    zs = np.where(keep, z.astype(np.float64), -np.inf)
    p = np.exp(zs - zs.max())
    p /= p.sum()
    if top_p < 1.0:
        order = np.argsort(-p, kind="stable")
        above = np.cumsum(p[order]) - p[order]
        drop = above >= top_p
        drop[0] = False
        keep[order[drop]] = False
    return keep, p


@pytest.mark.parametrize("dt,V,top_k,top_p", [(torch.float32, 151936, 50, 1.0), (torch.float32, 151936, 0, 0.9),
                                              (torch.bfloat16, 151936, 40, 0.8), (torch.float32, 1001, 0, 0.5),
                                              (torch.bfloat16, 1001, 3, 1.0), (torch.float32, 77, 7, 0.95)])
def test_top_k_top_p_sampling_matches_oracle(dt, V, top_k, top_p):
    """HF top-k / top-p: the sampled token is the oracle's exponential race over the HF-kept set (same Philox
    stream); a token at the cut boundary (ties or float32 mass rounding) may differ, never one far outside."""
    rng = np.random.default_rng(V + top_k)
    N = 64
    x = (rng.standard_normal((N, V)) * 2.5).astype(np.float32)
    logits = T(x).to(dt)
    xs = logits.float().cpu().numpy()
    out = torch.empty(N, dtype=torch.int64, device=DEV)
    seed, step, temp = 77, 5, 0.7
    native.select_tokens(logits, out, do_sample=True, temperature=temp, top_k=top_k, top_p=top_p, seed=seed, step=step)
    got = out.cpu().numpy()
    exact = 0
    for i in range(N):
        z = (xs[i] / np.float32(temp)).astype(np.float32)
        keep, p = _hf_kept(z, top_k, top_p)
        want = oracle.sample_row(xs[i], temp, top_k, top_p, seed, step, i)
        if got[i] == want:
            exact += 1
            continue
        # mismatch only when the drawn token sits at the cut: z within float32 rounding of the smallest kept z
        zmin = z[keep].min()
        assert abs(z[got[i]] - zmin) <= 1e-5 * max(1.0, abs(zmin)) or keep[got[i]], (i, got[i], want)
    assert exact >= N - 3, exact
    # deterministic across calls (integer-atomic histograms)
    out2 = torch.empty_like(out)
    native.select_tokens(logits, out2, do_sample=True, temperature=temp, top_k=top_k, top_p=top_p, seed=seed,
                         step=step)
    assert torch.equal(out, out2)


def test_top_p_distribution():
    """Nucleus draw frequencies: 8192 rows of the same logits, top_p = 0.8 keeps {0, 1, 2} (masses above them
    0, 0.46, 0.74 < 0.8; token 3 has 0.91 above) and renormalises."""
    z = torch.tensor([2.0, 1.5, 1.0, 0.0, -1.0, -2.0])
    N = 8192
    out = torch.empty(N, dtype=torch.int64, device=DEV)
    native.select_tokens(z.repeat(N, 1).to(DEV), out, do_sample=True, temperature=1.0, top_p=0.8, seed=5, step=1)
    freq = np.bincount(out.cpu().numpy(), minlength=6) / N
    p = torch.softmax(z, 0).numpy()
    keep, _ = _hf_kept(z.numpy(), 0, 0.8)
    assert keep.tolist() == [True, True, True, False, False, False]
    q = np.where(keep, p, 0)
    q /= q.sum()
    assert np.abs(freq - q).max() < 4 * np.sqrt(q.max() * (1 - q.max()) / N), (freq, q)
    assert freq[3:].sum() == 0


def test_sampling_distribution():
    """The race draw is softmax-distributed: 8192 rows of the same 6 logits, distinct Philox counters."""
    z = torch.tensor([2.0, 1.0, 0.5, 0.0, -1.0, -30.0])
    N = 8192
    logits = z.repeat(N, 1).to(DEV)
    out = torch.empty(N, dtype=torch.int64, device=DEV)
    native.select_tokens(logits, out, do_sample=True, temperature=1.0, seed=99, step=3)
    freq = np.bincount(out.cpu().numpy(), minlength=6) / N
    p = torch.softmax(z, 0).numpy()
    assert np.abs(freq - p).max() < 4 * np.sqrt(p.max() * (1 - p.max()) / N), (freq, p)
    assert freq[5] == 0


@pytest.mark.parametrize("V", [151936, 4099])
def test_greedy_sliced_ties_and_nan(V):
    """Greedy across workgroup slices keeps torch.argmax semantics: first index on ties (also across
    slice boundaries), NaN is the maximum, -inf rows pick index 0; unaligned fp32 rows (scalar path)."""
    N = 6
    x = torch.randn(N, V + 1, device=DEV)[:, :V]  # row stride V+1: unaligned rows for fp32
    x[0, V - 1] = 50.0
    x[0, 3] = 50.0  # tie: first index wins
    x[1, V // 2 + 1] = float("nan")
    x[1, V - 2] = float("nan")
    x[2] = float("-inf")
    x[3, V - 1] = 1e30
    out = torch.empty(N, dtype=torch.int64, device=DEV)
    for t in (x, x.to(torch.bfloat16)):
        native.select_tokens(t, out)
        want = torch.argmax(t.float(), -1)
        assert out.tolist() == want.tolist()
        assert out[0].item() == 3 and out[1].item() == V // 2 + 1


# ---------------------------------------------------------------------------------------------------- A15
def test_adamw_clip_matches_torch():
    torch.manual_seed(0)
    n = 1_000_003
    p0 = torch.randn(n, device=DEV)
    grads = [torch.randn(n, device=DEV) * s for s in (3.0, 0.01)]
    ref = p0.clone().requires_grad_(True)
    opt = torch.optim.AdamW([ref], lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2)
    p = p0.clone()
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    pbf = torch.empty(n, dtype=torch.bfloat16, device=DEV)
    for step, g in enumerate(grads, start=1):
        ref.grad = g.clone()
        tn = torch.nn.utils.clip_grad_norm_([ref], max_norm=1.0)
        opt.step()
        nrm = native.grad_norm(g)
        torch.testing.assert_close(nrm[0], tn, rtol=1e-5, atol=0)
        native.adamw_step(p, g, m, v, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=1e-2, step=step,
                          max_grad_norm=1.0, grad_norm_t=nrm, params_bf16=pbf)
        torch.testing.assert_close(p, ref.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(pbf.float(), p, rtol=1e-2, atol=0)


def test_adamw_skips_non_finite_norm():
    p = torch.ones(1000, device=DEV)
    g = torch.ones(1000, device=DEV)
    g[10] = float("inf")
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    nrm = native.grad_norm(g)
    native.adamw_step(p, g, m, v, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=1e-2, step=1,
                      max_grad_norm=1.0, grad_norm_t=nrm)
    assert torch.equal(p, torch.ones_like(p)) and torch.equal(m, torch.zeros_like(m))
