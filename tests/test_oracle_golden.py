"""Pin the CPU oracle against golden vectors produced by the reference itself (tests/golden/make_golden.py).

CPU-only: these run in the build container and on the GPU box alike (no reference needed at run time).
"""

import numpy as np
import pytest

import oracle

LOSS_KEYS = ["pg_loss", "pg_clipfrac", "ppo_kl", "pg_clipfrac_lower", "entropy_loss", "kl_loss", "loss"]


def test_ppo_actor_loss_matches_reference(golden):
    z, meta = golden("ppo_loss.npz")
    for ci, cfg in enumerate(meta["cases"]):
        g = lambda k: z[f"c{ci}_{k}"]  # noqa: E731
        out = oracle.actor_loss(
            g("old_log_prob"), g("log_prob"), g("advantages"), g("response_mask"), g("entropy"), g("ref_log_prob"),
            loss_agg_mode=cfg["loss_agg_mode"], clip_ratio_low=cfg["clip_ratio_low"],
            clip_ratio_high=cfg["clip_ratio_high"], clip_ratio_c=cfg["clip_ratio_c"],
            entropy_coeff=cfg["entropy_coeff"], use_kl_loss=cfg["use_kl_loss"], kl_loss_type=cfg["kl_loss_type"],
            kl_loss_coef=cfg["kl_loss_coef"], loss_scale_factor=cfg["loss_scale_factor"])
        amb = oracle.clip_boundary_tokens(g("old_log_prob"), g("log_prob"), g("advantages"), g("response_mask"),
                                          cfg["clip_ratio_low"], cfg["clip_ratio_high"], cfg["clip_ratio_c"])
        count = max(int(g("response_mask").sum()), 1)
        for k in LOSS_KEYS:
            atol = 1e-6 + (amb / count if "clipfrac" in k else 0.0)
            np.testing.assert_allclose(out[k], g(f"out_{k}"), rtol=2e-5, atol=atol, err_msg=f"case {ci} {k} {cfg}")
        np.testing.assert_allclose(out["dlogp"], g("out_dlogp"), rtol=1e-4, atol=1e-9, err_msg=f"case {ci} dlogp")
        np.testing.assert_allclose(out["dentropy"], g("out_dentropy"), rtol=1e-5, atol=1e-10, err_msg=f"case {ci} dent")
        np.testing.assert_allclose(out["kld"], g("out_kld"), rtol=1e-5, atol=1e-6, err_msg=f"case {ci} kld")


def test_gpg_actor_loss_matches_reference(golden):
    z, meta = golden("gpg_loss.npz")
    for ci, c in enumerate(meta["cases"]):
        g = lambda k: z[f"c{ci}_{k}"]  # noqa: E731
        r = oracle.actor_loss(g("old_log_prob"), g("log_prob"), g("advantages"), g("response_mask"), g("entropy"),
                              g("ref_log_prob"), clip_ratio_low=0.2, clip_ratio_high=0.2, clip_ratio_c=3.0,
                              policy_loss="gpg", **c)
        np.testing.assert_allclose(r["pg_loss"], g("out_pg_loss"), rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(r["loss"], g("out_loss"), rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(r["dlogp"], g("out_dlogp"), rtol=2e-5, atol=1e-9)
        np.testing.assert_allclose(r["dentropy"], g("out_dentropy"), rtol=2e-5, atol=1e-9)
        assert (g("out_clip") == 0).all()


def test_gspo_geo_mean_actor_loss_matches_reference(golden):
    """The oracle's GSPO / GMPO restatements composed as dp_actor does, against the reference's autograd."""
    z, meta = golden("seq_loss.npz")
    for ci, c in enumerate(meta["cases"]):
        g = lambda k: z[f"c{ci}_{k}"]  # noqa: E731
        want = oracle.actor_loss(g("old_log_prob"), g("log_prob"), g("advantages"), g("response_mask"), g("entropy"),
                                 g("ref_log_prob"), loss_agg_mode=c["loss_agg_mode"], clip_ratio_low=c["clip_ratio_low"],
                                 clip_ratio_high=c["clip_ratio_high"], clip_ratio_c=3.0, entropy_coeff=c["entropy_coeff"],
                                 use_kl_loss=True, kl_loss_type=c["kl_loss_type"], kl_loss_coef=c["kl_loss_coef"],
                                 loss_scale_factor=c["loss_scale_factor"], policy_loss=c["policy_loss"])
        np.testing.assert_allclose(want["pg_loss"], g("out_pg_loss"), rtol=2e-5, atol=1e-6, err_msg=str(c))
        np.testing.assert_allclose(want["loss"], g("out_loss"), rtol=2e-5, atol=1e-6, err_msg=str(c))
        np.testing.assert_allclose([want["pg_clipfrac"], want["ppo_kl"], want["pg_clipfrac_lower"]], g("out_clip"),
                                   rtol=2e-5, atol=1e-6, err_msg=str(c))
        d = g("out_dlogp")
        np.testing.assert_allclose(want["dlogp"], d, rtol=2e-4, atol=1e-6 * np.abs(d).max(), err_msg=str(c))
        np.testing.assert_allclose(want["dentropy"], g("out_dentropy"), rtol=1e-5, atol=1e-9, err_msg=str(c))


def test_cov_actor_loss_matches_reference(golden):
    """The oracle's Clip-Cov / KL-Cov restatements composed as dp_actor does, against the reference's autograd
    (clip_cov in the regime where every candidate is taken: the reference's subset draw is torch.randperm)."""
    z, meta = golden("cov_loss.npz")
    for ci, c in enumerate(meta["cases"]):
        g = lambda k: z[f"c{ci}_{k}"]  # noqa: E731
        want = oracle.actor_loss(g("old_log_prob"), g("log_prob"), g("advantages"), g("response_mask"), g("entropy"),
                                 g("ref_log_prob"), loss_agg_mode=c["loss_agg_mode"], clip_ratio_low=c["clip_ratio_low"],
                                 clip_ratio_high=c["clip_ratio_high"], clip_ratio_c=3.0, entropy_coeff=c["entropy_coeff"],
                                 use_kl_loss=True, kl_loss_type=c["kl_loss_type"], kl_loss_coef=c["kl_loss_coef"],
                                 loss_scale_factor=c["loss_scale_factor"], policy_loss=c["policy_loss"],
                                 cov_ratio=c["cov_ratio"], clip_cov_lb=c["clip_cov_lb"], clip_cov_ub=c["clip_cov_ub"],
                                 ppo_kl_coef=c["ppo_kl_coef"])
        np.testing.assert_allclose(want["pg_loss"], g("out_pg_loss"), rtol=2e-5, atol=1e-6, err_msg=str(c))
        np.testing.assert_allclose(want["loss"], g("out_loss"), rtol=2e-5, atol=1e-6, err_msg=str(c))
        np.testing.assert_allclose([want["pg_clipfrac"], want["ppo_kl"], want["pg_clipfrac_lower"]], g("out_clip"),
                                   rtol=2e-5, atol=1e-6, err_msg=str(c))
        d = g("out_dlogp")
        np.testing.assert_allclose(want["dlogp"], d, rtol=2e-4, atol=1e-6 * np.abs(d).max(), err_msg=str(c))


def test_masked_mean_known_answers(golden):
    z, _ = golden("masked_mean.npz")
    # tests/utils/test_torch_functional.py:55-66 — NaN outside the mask is ignored
    np.testing.assert_allclose(oracle.masked_mean(z["kat_values"], z["kat_mask"]), z["kat_out"], rtol=1e-6)
    np.testing.assert_allclose(oracle.masked_mean(z["kat_values"], z["kat_mask"]), 7.0 / 3.0, rtol=1e-6)
    np.testing.assert_allclose(oracle.masked_mean(z["rand_values"], z["rand_mask"]), z["rand_out_all"], rtol=1e-5)
    np.testing.assert_allclose(oracle.masked_mean(z["rand_values"], z["rand_mask"], axis=1), z["rand_out_axis1"], rtol=1e-5)
    np.testing.assert_allclose(oracle.masked_var(z["rand_values"], z["rand_mask"]), z["rand_var"], rtol=1e-5)
    np.testing.assert_allclose(oracle.masked_whiten(z["rand_values"], z["rand_mask"]), z["rand_whiten"], rtol=1e-5, atol=1e-6)


def test_grpo_matches_reference(golden):
    z, meta = golden("grpo.npz")
    for ci, cfg in enumerate(meta["cases"]):
        adv, ret = oracle.grpo_outcome_advantage(z[f"c{ci}_rewards"], z[f"c{ci}_mask"], list(z[f"c{ci}_uid"]),
                                                 cfg["epsilon"], cfg["norm_adv_by_std_in_grpo"])
        np.testing.assert_allclose(adv, z[f"c{ci}_adv"], rtol=2e-5, atol=2e-6, err_msg=str(cfg))
        np.testing.assert_allclose(ret, z[f"c{ci}_ret"], rtol=2e-5, atol=2e-6, err_msg=str(cfg))


def test_rloo_and_reinforce_pp_baseline_match_reference(golden):
    z, meta = golden("group_adv.npz")
    fns = {"rloo": oracle.rloo_outcome_advantage, "reinforce_plus_plus_baseline": oracle.reinforce_pp_baseline_outcome_advantage}
    for ci, c in enumerate(meta["cases"]):
        adv, ret = fns[c["estimator"]](z[f"c{ci}_rewards"], z[f"c{ci}_mask"], list(z[f"c{ci}_uid"]))
        np.testing.assert_allclose(adv, z[f"c{ci}_adv"], rtol=2e-5, atol=2e-6, err_msg=str(c))
        np.testing.assert_allclose(ret, z[f"c{ci}_ret"], rtol=2e-5, atol=2e-6, err_msg=str(c))


def _more_adv_oracle(z, ci, est):
    r, m, uid = z[f"c{ci}_rewards"], z[f"c{ci}_mask"], list(z[f"c{ci}_uid"]) if f"c{ci}_uid" in z else None
    if est == "opo":
        return oracle.opo_outcome_advantage(r, m, uid)
    if est == "gpg":
        return oracle.gpg_outcome_advantage(r, m, uid)
    if est == "remax":
        return oracle.remax_advantage_return(r, z[f"c{ci}_baselines"], m)
    return oracle.grpo_passk_outcome_advantage(r, m, uid, norm_adv_by_std_in_grpo=est.endswith("_std"))


def test_opo_gpg_passk_remax_match_reference(golden):
    """The oracle's OPO / GPG / GRPO pass@k / ReMax restatements against the reference's estimators."""
    z, meta = golden("more_adv.npz")
    for ci, c in enumerate(meta["cases"]):
        adv, ret = _more_adv_oracle(z, ci, c["estimator"])
        np.testing.assert_allclose(adv, z[f"c{ci}_adv"], rtol=2e-5, atol=2e-6, err_msg=str(c))
        np.testing.assert_allclose(ret, z[f"c{ci}_ret"], rtol=2e-5, atol=2e-6, err_msg=str(c))
    with pytest.raises(ValueError) as e:
        oracle.grpo_passk_outcome_advantage(np.ones((3, 4)), np.ones((3, 4)), ["a", "a", "b"])
    assert str(e.value) == meta["passk_singleton_error"]


def test_reinforce_pp_matches_reference(golden):
    z, meta = golden("rfpp.npz")
    for ci, c in enumerate(meta["cases"]):
        adv, ret = oracle.reinforce_pp_advantage_return(z[f"c{ci}_rewards"], z[f"c{ci}_mask"], c["gamma"])
        np.testing.assert_allclose(adv, z[f"c{ci}_adv"], rtol=2e-5, atol=2e-6)
        np.testing.assert_allclose(ret, z[f"c{ci}_ret"], rtol=1e-6, atol=1e-7)


def test_gae_matches_reference(golden):
    z, meta = golden("gae.npz")
    for ci, cfg in enumerate(meta["cases"]):
        adv, ret = oracle.gae_advantage_return(z[f"c{ci}_rewards"], z[f"c{ci}_values"], z[f"c{ci}_mask"],
                                               cfg["gamma"], cfg["lam"])
        np.testing.assert_allclose(adv, z[f"c{ci}_adv"], rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(ret, z[f"c{ci}_ret"], rtol=1e-5, atol=1e-5)


def test_gae_bf16_values_matches_reference(golden):
    """GAE over bf16 critic values: the reference rounds gamma * V(t+1) to bf16 (bf16 tensor arithmetic)."""
    z, meta = golden("gae_bf16.npz")
    for ci, cfg in enumerate(meta["cases"]):
        adv, ret = oracle.gae_advantage_return(z[f"c{ci}_rewards"], z[f"c{ci}_values"], z[f"c{ci}_mask"],
                                               cfg["gamma"], cfg["lam"], values_bf16=True)
        np.testing.assert_allclose(adv, z[f"c{ci}_adv"], rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(ret, z[f"c{ci}_ret"], rtol=1e-5, atol=1e-5)


def test_value_loss_matches_reference(golden):
    """compute_value_loss (core_algos.py:1230-1269) fwd + d/d vpreds, fp32 and bf16 critic outputs, 4 agg modes,
    vpreds on the clip bounds. bf16: the reference's vpreds gradient is itself a bf16 tensor (one rounding)."""
    z, meta = golden("value_loss.npz")
    assert len(meta["cases"]) == 16
    for ci, cfg in enumerate(meta["cases"]):
        bf = cfg["dtype"] == "bfloat16"
        vf, cf, vm, dv = oracle.value_loss(z[f"c{ci}_vpreds"], z[f"c{ci}_values"], z[f"c{ci}_returns"], z[f"c{ci}_mask"],
                                           cfg["cliprange_value"], cfg["mode"], cfg["loss_scale_factor"], value_bf16=bf)
        np.testing.assert_allclose(vf, z[f"c{ci}_vf_loss"], rtol=3e-5, err_msg=str(cfg))  # fp32 sum order
        np.testing.assert_allclose(cf, z[f"c{ci}_vf_clipfrac"], rtol=1e-6, atol=1e-7, err_msg=str(cfg))
        np.testing.assert_allclose(vm, z[f"c{ci}_vpred_mean"], rtol=1e-5, atol=1e-6, err_msg=str(cfg))
        ref = z[f"c{ci}_dvpreds"]
        if bf:
            dv = oracle.bf16_round(dv)
            np.testing.assert_allclose(dv, ref, rtol=8e-3, atol=1e-3 * np.abs(ref).max(), err_msg=str(cfg))
        else:
            np.testing.assert_allclose(dv, ref, rtol=2e-5, atol=1e-7 * np.abs(ref).max(), err_msg=str(cfg))


def regen_logits(case):
    rng = np.random.default_rng(case["seed"])
    x = (rng.standard_normal((case["N"], case["V"]), dtype=np.float32) * np.float32(case["scale"])).astype(np.float32)
    labels = rng.integers(0, case["V"], size=(case["N"],), dtype=np.int64)
    dlogp = rng.standard_normal((case["N"],), dtype=np.float32)
    dent = rng.standard_normal((case["N"],), dtype=np.float32)
    return x, labels, dlogp, dent


def bf16_round(x):
    u = np.asarray(x, np.float32).view(np.uint32).astype(np.uint64)
    u = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return u.astype(np.uint32).view(np.float32)


@pytest.mark.parametrize("ci", [0, 1, 2, 3])
def test_logprob_entropy_matches_reference(golden, ci):
    z, meta = golden("logprob.npz")
    case = meta["cases"][ci]
    x, labels, dlogp, dent = regen_logits(case)
    import hashlib
    assert hashlib.sha256(x.tobytes()).hexdigest() == str(z[f"c{ci}_sha256"])
    for dt in ("fp32", "bf16"):
        xin = x if dt == "fp32" else bf16_round(x)
        logp, ent, _ = oracle.logprob_entropy(xin, labels)
        np.testing.assert_allclose(logp, z[f"c{ci}_{dt}_logp"], rtol=1e-5, atol=2e-5)
        # the reference sums 151936 float32 terms: its own rounding is ~1e-5 relative
        np.testing.assert_allclose(ent, z[f"c{ci}_{dt}_entropy"], rtol=5e-5, atol=2e-5)
        g_lp = oracle.logprob_entropy_backward(xin, labels, dlogp, np.zeros_like(dent))
        g_ent = oracle.logprob_entropy_backward(xin, labels, np.zeros_like(dlogp), dent)
        if case["inputs_from_seed"]:
            idx = np.arange(0, x.size, 997)
            np.testing.assert_allclose(g_lp.reshape(-1)[idx], z[f"c{ci}_{dt}_dlogits_lp_sample"], rtol=1e-4, atol=1e-9)
            np.testing.assert_allclose(g_ent.reshape(-1)[idx], z[f"c{ci}_{dt}_dlogits_ent_sample"], rtol=1e-3, atol=1e-9)
            np.testing.assert_allclose(np.abs(g_lp).sum(-1), z[f"c{ci}_{dt}_dlogits_lp_rowsum_abs"], rtol=1e-4)
        else:
            np.testing.assert_allclose(g_lp, z[f"c{ci}_{dt}_dlogits_lp"], rtol=1e-4, atol=1e-8)
            np.testing.assert_allclose(g_ent, z[f"c{ci}_{dt}_dlogits_ent"], rtol=1e-3, atol=1e-7)
        if dt == "bf16":
            # the reference's bf16 path rounds its output to bf16; ours stays fp32: equal up to that rounding
            np.testing.assert_allclose(logp, z[f"c{ci}_{dt}_logp_refbf16"], rtol=1e-2, atol=0.07)


def test_fused_linear_matches_reference(golden):
    z, meta = golden("fused_linear.npz")
    for ci, cfg in enumerate(meta["cases"]):
        g = lambda k: z[f"c{ci}_{k}"]  # noqa: E731
        lp, ent = oracle.fused_linear_logprob_entropy(g("hidden"), g("weight"), g("input_ids"), cfg["temperature"])
        np.testing.assert_allclose(lp, g("out_logp"), rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(ent, g("out_entropy"), rtol=1e-5, atol=1e-5)
        dh, dw = oracle.fused_linear_backward(g("hidden"), g("weight"), g("input_ids"), g("dlogp"), g("dentropy"),
                                              cfg["temperature"])
        np.testing.assert_allclose(dh, g("out_dhidden"), rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(dw, g("out_dweight"), rtol=1e-4, atol=1e-5)


def test_masks_and_positions_match_reference(golden):
    z, _ = golden("masks.npz")
    np.testing.assert_array_equal(oracle.get_response_mask(z["doc_responses"], 1), z["doc_mask_eos1"])
    np.testing.assert_array_equal(oracle.get_response_mask(z["doc_responses"], [1, 2]), z["doc_mask_eos12"])
    np.testing.assert_array_equal(oracle.get_response_mask(z["rand_responses"], 7), z["rand_mask_eos7"])
    np.testing.assert_array_equal(oracle.get_response_mask(z["rand_responses"], [7, 9, 11]), z["rand_mask_eos7_9_11"])
    np.testing.assert_array_equal(oracle.compute_position_id_with_mask(z["prompt_attention_mask"]), z["prompt_position_ids"])
    R = z["full_position_ids"].shape[1] - z["prompt_position_ids"].shape[1]
    np.testing.assert_array_equal(oracle.response_position_ids(z["prompt_position_ids"], R), z["full_position_ids"])


def test_greedy_first_index_tie_break():
    # torch.argmax semantics the reference relies on (argmax([3,3,1]) == 0)
    assert oracle.greedy(np.array([[3.0, 3.0, 1.0], [0.0, 1.0, 1.0]])).tolist() == [0, 1]


def _tiny_cfg_and_params(name="tiny_qwen2"):
    import json
    import os
    import types

    import torch
    from safetensors.torch import load_file

    from oracle import qwen2_ref

    d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", name)
    c = json.load(open(os.path.join(d, "config.json")))
    cfg = types.SimpleNamespace(**c)
    cfg.head_dim = cfg.hidden_size // cfg.num_attention_heads
    return cfg, qwen2_ref.load_hf_state_dict(cfg, load_file(os.path.join(d, "model.safetensors")))


def test_qwen2_restatement_matches_reference_model(golden):
    """oracle.qwen2_ref (the CPU model used by GPU parity tests and the CPU baseline) reproduces the
    reference's HF model: greedy rollout tokens bit-exact, log-probs / entropy to fp32 rounding."""
    import torch

    from oracle import qwen2_ref

    z, meta = golden("tiny_qwen2_rollout.npz")
    cfg, P = _tiny_cfg_and_params()
    t = lambda k: torch.from_numpy(np.ascontiguousarray(z[k]))  # noqa: E731
    resp = qwen2_ref.generate_greedy(cfg, P, t("prompt_ids"), t("prompt_attention_mask"), t("prompt_position_ids"),
                                     meta["response_length"], [meta["eos_token_id"]], meta["pad_token_id"])
    np.testing.assert_array_equal(resp.numpy(), z["responses"])
    ids, am, pos, r = t("sequences"), t("attention_mask"), t("position_ids"), t("responses")
    lp, ent = qwen2_ref.logp_entropy(cfg, P, ids, am, pos, r)
    np.testing.assert_allclose(lp.numpy(), z["log_probs"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(ent.numpy(), z["entropy"], rtol=1e-5, atol=1e-5)
    lp7, _ = qwen2_ref.logp_entropy(cfg, P, ids, am, pos, r, temperature=0.7)
    np.testing.assert_allclose(lp7.numpy(), z["log_probs_t07"], rtol=1e-5, atol=1e-5)


def test_llama_restatement_matches_reference_model(golden):
    """The same restatement with attention_bias=False / untied lm_head / head_dim 128 / rope_theta 5e5
    reproduces HF LlamaForCausalLM (config #4's architecture): greedy tokens bit-exact, log-probs to fp32."""
    import torch

    from oracle import qwen2_ref

    z, meta = golden("tiny_llama_rollout.npz")
    cfg, P = _tiny_cfg_and_params("tiny_llama")
    assert cfg.head_dim == 128 and not cfg.attention_bias and "layers.0.qkv_proj.bias" not in P
    t = lambda k: torch.from_numpy(np.ascontiguousarray(z[k]))  # noqa: E731
    resp = qwen2_ref.generate_greedy(cfg, P, t("prompt_ids"), t("prompt_attention_mask"), t("prompt_position_ids"),
                                     meta["response_length"], [meta["eos_token_id"]], meta["pad_token_id"])
    np.testing.assert_array_equal(resp.numpy(), z["responses"])
    lp, ent = qwen2_ref.logp_entropy(cfg, P, t("sequences"), t("attention_mask"), t("position_ids"), t("responses"))
    np.testing.assert_allclose(lp.numpy(), z["log_probs"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(ent.numpy(), z["entropy"], rtol=1e-5, atol=1e-5)
