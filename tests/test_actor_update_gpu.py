"""Reference-pinned actor update and GRPO step (SURVEY §8(c) golden #7; VERDICT r01 "missing" 1 and 2).

Fixtures (tests/golden/make_golden.py, fp32 reference runs on the committed tiny Qwen2 weights):

* ``actor_update.npz``: the reference DataParallelPPOActor.compute_log_prob + update_policy (dp_actor.py:300-482)
  with torch AdamW + clip_grad_norm_ (fsdp_workers.py:454-459, dp_actor.py:282-298), 2 mini-batches x 2
  micro-batches, noisy old log-probs (ratios across the clip bounds), +- advantages; two configs (GRPO's k3 KL
  token-mean; entropy bonus + seq-mean-token-mean + k1 KL + clip-higher + dual-clip c=10).
* ``grpo_step.npz``: one fit() step composed from the reference's functions (ray_trainer.py:1104-1399): HFRollout
  greedy -> response mask -> reward-model scores through NaiveRewardManager -> old log-prob + entropy -> ref
  log-prob -> compute_advantage(GRPO) -> update_policy -> step metrics; n = 2 (real groups) and n = 1.

Here the same inputs go through this repository's HIP path in fp32 (compute_dtype=float32) on the GPU.
Tolerances: log-probs / entropy 1e-4 (the model-level bar of test_model_gpu.py); loss and KL metrics 1e-4
absolute; grad norms 1e-4 relative; per-tensor parameter sums after the update 1e-5 relative; the update
itself (after - before) within 2 % of its own size for 99.9 % of the elements (AdamW's first steps move an
element by ~lr * sign(g), so elements whose gradient is at fp32 noise level may legitimately flip).
"""

import json
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
TINY = os.path.join(HERE, "golden", "tiny_qwen2")
sys.path.insert(0, os.path.join(HERE, "golden"))


def T(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _fixture(name):
    z = np.load(os.path.join(HERE, "golden", name), allow_pickle=False)
    return z, json.loads(str(z["__meta__"]))


def _tiny(trainable=True):
    from safetensors.torch import load_file

    from dots.rl_amd.qwen2 import ParamStore, Qwen2Config, Qwen2Model

    cfg = Qwen2Config.from_dict(json.load(open(os.path.join(TINY, "config.json"))))
    store = ParamStore(cfg, "cuda", compute_dtype=torch.float32, trainable=trainable)
    store.load_state_dict_hf(load_file(os.path.join(TINY, "model.safetensors")))
    return cfg, store, Qwen2Model(cfg, store)


def _ref_after_master(cfg, z, prefix):
    """The reference's post-step HF state dict mapped into this repository's flat fused layout (on the CPU)."""
    from dots.rl_amd.qwen2 import ParamStore

    sd = {k[len(prefix) + len("after."):]: torch.from_numpy(z[k]) for k in z.files if k.startswith(prefix + "after.")}
    ref = ParamStore(cfg, "cpu", compute_dtype=torch.float32, trainable=False)
    ref.load_state_dict_hf(sd)
    return ref, sd


def _check_params(cfg, store, before, z, prefix, param_sums):
    ref, sd = _ref_after_master(cfg, z, prefix)
    # per-tensor sums of the post-step parameters (HF names)
    got_sd = {}
    H = cfg.hidden_size
    for name, (o, shape, _) in store.offsets.items():
        got_sd[name] = store.master[o:o + int(np.prod(shape))].view(shape).double().cpu()
    for k, want in param_sums.items():
        if k == "model.embed_tokens.weight":
            got = got_sd["embed_tokens"].sum().item()
        elif k == "model.norm.weight":
            got = got_sd["norm"].sum().item()
        else:
            i = int(k.split(".")[2])
            p = f"layers.{i}."
            if "input_layernorm" in k:
                got = got_sd[p + "input_layernorm"].sum().item()
            elif "post_attention_layernorm" in k:
                got = got_sd[p + "post_attention_layernorm"].sum().item()
            elif "o_proj" in k:
                got = got_sd[p + "o_proj"].sum().item()
            elif "down_proj" in k:
                got = got_sd[p + "down_proj"].sum().item()
            elif "gate_proj" in k or "up_proj" in k:
                gu = got_sd[p + "gate_up_proj"]
                I = gu.shape[0] // 2
                got = (gu[:I] if "gate_proj" in k else gu[I:]).sum().item()
            else:  # q/k/v weight or bias
                nq, nkv = cfg.num_attention_heads * cfg.head_dim, cfg.num_key_value_heads * cfg.head_dim
                t = got_sd[p + ("qkv_proj.bias" if k.endswith("bias") else "qkv_proj.weight")]
                rng = {"q_proj": (0, nq), "k_proj": (nq, nq + nkv), "v_proj": (nq + nkv, nq + 2 * nkv)}
                a, b = next(v for x, v in rng.items() if x in k)
                got = t[a:b].sum().item()
        scale = max(abs(want), float(np.abs(sd[k].double().numpy()).sum()) * 1e-3)
        assert abs(got - want) <= 1e-5 * scale, (k, got, want)
    # the update itself, element by element
    after = store.master.detach().cpu()
    d_got = (after - before).numpy()
    d_ref = (ref.master - before).numpy()
    step = np.abs(d_ref)
    bad = np.abs(d_got - d_ref) > 0.02 * np.maximum(step, np.median(step[step > 0]))
    assert bad.mean() < 1e-3, f"{bad.sum()} of {bad.size} parameter updates differ from the reference"
    assert np.abs(d_ref).sum() > 0


def _metric_lists_close(got, want):
    assert set(got) >= set(want), set(want) - set(got)
    for k, ref in want.items():
        g = np.asarray(got[k], dtype=np.float64)
        r = np.asarray(ref, dtype=np.float64)
        assert g.shape == r.shape, (k, g.shape, r.shape)
        if k == "actor/grad_norm":
            np.testing.assert_allclose(g, r, rtol=1e-4, err_msg=k)
        elif "clipfrac" in k:  # a token exactly on a clip bound may land either side in a different fp32 order
            np.testing.assert_allclose(g, r, atol=0.051, err_msg=k)
        else:
            np.testing.assert_allclose(g, r, rtol=1e-4, atol=1e-4, err_msg=k)


@pytest.mark.parametrize("exec_mb", [1, 0])
@pytest.mark.parametrize("ci", [0, 1])
def test_update_policy_matches_reference(ci, exec_mb):
    """exec_mb = 1: one micro-batch per forward / backward as the reference; 0 (auto): both micro-batches of a
    mini-batch in one pass with their losses kept per micro-batch — the same fixture, the same tolerances."""
    from dots.rl_amd.config import to_attr
    from dots.rl_amd.dp_actor import DataParallelPPOActor, FlatAdamW
    from dots.rl_amd.protocol import DataProto

    z, meta = _fixture("actor_update.npz")
    case = meta["cases"][ci]
    c = lambda k: T(z[f"c{ci}_{k}"])  # noqa: E731
    cfg, store, model = _tiny()
    before = store.master.detach().cpu().clone()
    acfg = to_attr(dict(case["config"], exec_micro_batches=exec_mb))
    opt = FlatAdamW(store, lr=case["lr"], betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01,
                    max_grad_norm=acfg.grad_clip)
    actor = DataParallelPPOActor(acfg, model, opt)
    data = DataProto.from_dict({k: c(k) for k in ("input_ids", "attention_mask", "position_ids", "responses")},
                               meta_info={"micro_batch_size": 4, "temperature": 1.0, "use_dynamic_bsz": False})
    lp, ent = actor.compute_log_prob(data, calculate_entropy=True)
    np.testing.assert_allclose(lp.cpu().numpy(), z[f"c{ci}_log_probs"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(ent.cpu().numpy(), z[f"c{ci}_entropys"], rtol=1e-4, atol=1e-4)
    udata = DataProto.from_dict({k: c(k) for k in ("input_ids", "attention_mask", "position_ids", "responses",
                                                   "response_mask", "old_log_probs", "advantages", "ref_log_prob")},
                                meta_info={"temperature": 1.0})
    metrics = actor.update_policy(udata)
    _metric_lists_close(metrics, case["metrics"])
    _check_params(cfg, store, before, z, f"c{ci}_", case["param_sums"])


class _PresetRM:
    """Reward-model worker group stand-in: preset per-row scores at the last valid response token (what the
    reference's rm_wg.compute_rm_score returns as rm_scores, ray_trainer.py:1200-1203)."""

    def __init__(self, scores):
        self.scores = scores

    def compute_rm_score(self, batch):
        from dots.rl_amd.protocol import DataProto

        R = batch.batch["responses"].shape[1]
        vl = batch.batch["attention_mask"][:, -R:].sum(-1)
        rm = torch.zeros(vl.shape[0], R, device=vl.device)
        rm[torch.arange(vl.shape[0], device=vl.device), vl - 1] = torch.tensor(self.scores, device=vl.device)
        return DataProto.from_dict({"rm_scores": rm})


@pytest.mark.parametrize("ci", [0, 1, 2])
def test_grpo_fit_step_matches_reference(ci):
    from stub_tokenizer import StubTokenizer

    from dots.rl_amd.config import apply_overrides, default_config
    from dots.rl_amd.reward import NaiveRewardManager
    from dots.rl_amd.trainer import RayPPOTrainer

    z, meta = _fixture("grpo_step.npz")
    m = meta["cases"][ci]
    Np, n, P, R = m["n_prompts"], m["n"], m["P"], m["R"]
    cfg = apply_overrides(default_config(), [
        f"data.train_batch_size={Np}", f"data.max_prompt_length={P}", f"data.max_response_length={R}",
        f"actor_rollout_ref.rollout.n={n}", f"actor_rollout_ref.rollout.response_length={R}",
        f"actor_rollout_ref.rollout.prompt_length={P}", "actor_rollout_ref.rollout.do_sample=False",
        f"actor_rollout_ref.actor.ppo_mini_batch_size={m['mini_prompts']}",
        f"actor_rollout_ref.actor.ppo_micro_batch_size_per_gpu={m['micro']}",
        "actor_rollout_ref.rollout.log_prob_micro_batch_size_per_gpu=4",
        "actor_rollout_ref.ref.log_prob_micro_batch_size_per_gpu=4", f"actor_rollout_ref.actor.optim.lr={m['lr']}",
        f"actor_rollout_ref.model.path={TINY}", "actor_rollout_ref.model.dtype=float32",
        "reward_model.enable=True", "reward_model.reward_manager=naive",
        "trainer.balance_batch=False", "algorithm.adv_estimator=grpo",
    ])
    trainer = RayPPOTrainer(cfg, tokenizer=StubTokenizer(), rm_wg=_PresetRM(m["rm_scores"]),
                            eos_token_id=m["eos_token_id"], pad_token_id=m["pad_token_id"])
    trainer.init_workers()
    if m.get("uid_pairs"):  # the reference case groups rows (2i, 2i + 1): distinct responses in one GRPO group
        trainer._uids = lambda k: np.array([f"pair{i // 2}" for i in range(k)], dtype=object)
    store = trainer.actor_rollout_wg.worker.store
    before = store.master.detach().cpu().clone()
    trainer.global_steps = 1
    gts = m["ground_truths"]
    batch_dict = {"input_ids": T(z[f"c{ci}_prompt_ids"]), "attention_mask": T(z[f"c{ci}_prompt_attention_mask"]),
                  "position_ids": T(z[f"c{ci}_prompt_position_ids"]),
                  "data_source": np.array(["openai/gsm8k"] * Np, dtype=object),
                  "reward_model": np.array([{"ground_truth": g} for g in gts], dtype=object)}
    metrics = trainer.step(batch_dict)
    b = trainer.last_batch
    for k in ("prompts", "responses", "input_ids", "attention_mask", "position_ids", "response_mask"):
        np.testing.assert_array_equal(b.batch[k].cpu().numpy(), z[f"c{ci}_{k}"], err_msg=k)
    np.testing.assert_array_equal(b.batch["token_level_scores"].cpu().numpy(), z[f"c{ci}_token_level_scores"])
    # the rule reward of the same responses (gsm8k strict through the naive manager) on the device batch
    b.batch.pop("rm_scores")
    rule = NaiveRewardManager(tokenizer=StubTokenizer(), num_examine=0)(b)
    np.testing.assert_array_equal(rule.cpu().numpy(), z[f"c{ci}_rule_scores"])
    for k in ("old_log_probs", "ref_log_prob"):
        np.testing.assert_allclose(b.batch[k].cpu().numpy(), z[f"c{ci}_{k}"], rtol=1e-4, atol=1e-4, err_msg=k)
    for k in ("advantages", "returns"):
        np.testing.assert_allclose(b.batch[k].cpu().numpy(), z[f"c{ci}_{k}"], rtol=1e-5, atol=1e-6, err_msg=k)
    np.testing.assert_allclose(metrics["actor/entropy"], m["actor_entropy"], rtol=1e-4)
    for k, v in m["data_metrics"].items():
        np.testing.assert_allclose(metrics[k], v, rtol=1e-5, atol=1e-6, err_msg=k)
    want = {k: float(np.mean(v)) for k, v in m["update_metrics"].items()}
    if not m["compare_update"]:
        # identical greedy group members with +-1/sqrt(2) advantages: the policy gradient cancels inside each
        # micro-batch (grad norm ~1e-7 in the reference), AdamW then moves every weight by ~lr along fp32 noise,
        # so only the pre-update quantities are comparable
        assert abs(metrics["actor/pg_loss"]) < 1e-6 and abs(want["actor/pg_loss"]) < 1e-6
        assert metrics["actor/pg_clipfrac"] == want["actor/pg_clipfrac"] == 0.0
        return
    for k, v in want.items():
        tol = dict(rtol=1e-4) if k == "actor/grad_norm" else dict(rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(metrics[k], v, err_msg=k, **tol)
    if m["compare_update"]:
        _check_params(trainer.actor_rollout_wg.worker.model_config, store, before, z, f"c{ci}_", m["param_sums"])
