"""Trainer steps with the registry's other advantage estimators (core_algos.py:327-684 via ray_trainer.py:214-291)
on a tiny random Qwen2: ReMax's greedy baseline rollout (ray_trainer.py:1160-1180), OPO, GPG, GRPO pass@k and
RLOO. The estimators themselves are pinned against the reference in test_kernels_gpu.py (more_adv.npz)."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

TINY = ("{'hidden_size': 128, 'intermediate_size': 256, 'num_hidden_layers': 2, 'num_attention_heads': 2, "
        "'num_key_value_heads': 1, 'vocab_size': 1024}")


def _trainer(estimator, extra=()):
    from dots.rl_amd.config import apply_overrides, default_config
    from dots.rl_amd.trainer import RayPPOTrainer

    cfg = apply_overrides(default_config(), [
        "data.train_batch_size=4", "data.max_prompt_length=32", "data.max_response_length=16",
        "actor_rollout_ref.rollout.n=4", "actor_rollout_ref.rollout.response_length=16",
        "actor_rollout_ref.rollout.prompt_length=32", "actor_rollout_ref.actor.ppo_mini_batch_size=2",
        "actor_rollout_ref.actor.ppo_micro_batch_size_per_gpu=4",
        "actor_rollout_ref.rollout.log_prob_micro_batch_size_per_gpu=8",
        "actor_rollout_ref.ref.log_prob_micro_batch_size_per_gpu=8", f"algorithm.adv_estimator={estimator}",
        f"actor_rollout_ref.model.override_config={TINY}", *extra,
    ])
    trainer = RayPPOTrainer(cfg)
    trainer.train_dataloader.vocab_limit = 1000
    trainer.init_workers()
    return trainer


@pytest.mark.parametrize("estimator", ["remax", "opo", "gpg", "grpo_passk", "rloo"])
def test_estimator_step_end_to_end(estimator):
    trainer = _trainer(estimator)
    m = trainer.fit(num_steps=1)[-1]
    for k in ["actor/pg_loss", "actor/grad_norm", "critic/advantages/mean", "critic/returns/mean"]:
        assert k in m and np.isfinite(m[k]), (k, m.get(k))
    b = trainer.last_batch.batch
    adv, ret, mask = b["advantages"], b["returns"], b["response_mask"]
    assert torch.isfinite(adv).all() and torch.isfinite(ret).all()
    assert (adv[mask == 0] == 0).all()
    if estimator == "remax":
        # ray_trainer.py:1160-1180: a greedy response per prompt scored by the reward function, its sum repeated
        # over the prompt's n samples; advantages = reverse-cumsum returns - baseline x mask
        assert "timing_s/gen_max" in m
        base = b["reward_baselines"]
        assert base.shape == (len(trainer.last_batch),)
        assert torch.equal(base.view(-1, 4), base.view(-1, 4)[:, :1].expand(-1, 4))
        r = (b["token_level_rewards"] * mask).flip(-1).cumsum(-1).flip(-1)
        torch.testing.assert_close(ret, r, rtol=1e-6, atol=1e-6)
        torch.testing.assert_close(adv, r - base[:, None] * mask, rtol=1e-6, atol=1e-6)
    if estimator == "grpo_passk":
        # one non-zero advantage row at most per group of n
        nz = (adv.abs().sum(-1) != 0).view(-1, 4).sum(-1)
        assert (nz <= 1).all()


@pytest.mark.parametrize("loss_mode", ["gspo", "geo_mean", "gpg", "clip_cov", "kl_cov"])
def test_policy_loss_modes_step_end_to_end(loss_mode):
    """actor.policy_loss.loss_mode selects the registered loss inside update_policy (dp_actor.py:419-466): one GRPO
    step per mode, finite metrics, the policy moves."""
    trainer = _trainer("grpo", [f"actor_rollout_ref.actor.policy_loss.loss_mode={loss_mode}"])
    w0 = trainer.actor_rollout_wg.worker.actor_store.master.clone() if hasattr(trainer.actor_rollout_wg, "worker") \
        and hasattr(trainer.actor_rollout_wg.worker, "actor_store") else None
    m = trainer.fit(num_steps=1)[-1]
    for k in ["actor/pg_loss", "actor/pg_clipfrac", "actor/ppo_kl", "actor/grad_norm"]:
        assert k in m and np.isfinite(m[k]), (k, m.get(k))
    if w0 is not None:
        assert not torch.equal(w0, trainer.actor_rollout_wg.worker.actor_store.master)



def test_update_step_bit_reproducible():
    """Two identical trainer steps (fresh trainers, same seeds) end with bit-identical parameters: every kernel of
    the update is deterministic, including the embedding backward (tied lm_head) and the weight gradients that run
    on a side stream concurrently with their input gradients."""
    masters = []
    for _ in range(2):
        trainer = _trainer("grpo", ["actor_rollout_ref.actor.use_kl_loss=True"])
        trainer.fit(num_steps=1)
        masters.append(trainer.actor_rollout_wg.worker.store.master.clone())
    assert torch.equal(masters[0], masters[1]), (masters[0] - masters[1]).abs().max().item()


def test_profile_step_records_the_hot_method_ranges(tmp_path):
    """start_profile / stop_profile around global_profiler.steps (ray_trainer.py:1096-1366) with the torch tool: the
    written trace holds the four annotated hot methods of the step (fsdp_workers.py:685,728,766,808) and their
    device kernels; a step outside the list writes nothing."""
    import json

    trainer = _trainer("grpo", ["global_profiler.steps=[2]", "actor_rollout_ref.actor.profiler.tool=torch",
                                "actor_rollout_ref.actor.profiler.enable=True",
                                "actor_rollout_ref.actor.profiler.all_ranks=True",
                                f"actor_rollout_ref.actor.profiler.save_path={tmp_path}"])
    trainer.fit(num_steps=2)
    prof = trainer.actor_rollout_wg.worker.profiler
    assert prof.traces == [str(tmp_path / "prof_step_2_rank_0.json")]
    with open(prof.traces[0]) as f:
        ev = json.load(f)["traceEvents"]
    names = {e.get("name") for e in ev}
    assert {"generate_sequences", "compute_log_prob", "compute_ref_log_prob", "update_actor"} <= names, names
    assert any(str(e.get("name", "")).startswith("void drl::") or "drl::" in str(e.get("name", "")) for e in ev
               if e.get("cat") == "kernel"), "no HIP kernel of this package in the trace"
