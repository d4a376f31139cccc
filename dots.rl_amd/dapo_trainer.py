"""DAPO recipe trainer (mirror of recipe/dapo/dapo_ray_trainer.py:60-370) on the SPMD single controller.

DAPO = the PPO step of ``RayPPOTrainer`` with: decoupled clip (clip_ratio_low 0.2 / clip_ratio_high 0.28,
fused in K1), token-mean aggregation, the overlong-buffer reward (``reward.DAPOSyntheticRewardManager``) and
dynamic sampling — generation batches are scored and filtered to prompt groups whose metric
(``seq_final_reward`` / ``seq_reward``) has non-zero spread (np.std > 0, or a single sample), accumulated
until ``data.train_batch_size`` prompts survive, then cut to ``train_batch_size * n`` trajectories
(dapo_ray_trainer.py:207-251). Everything after the filter is the PPO step's ``_train_on``.
"""

from __future__ import annotations

from collections import defaultdict

import numpy as np

from .protocol import DataProto
from .reward import DAPOSyntheticRewardManager, compute_reward
from .trainer import RayPPOTrainer, marked_timer


def filter_groups(batch: DataProto, metric_name: str):
    """dapo_ray_trainer.py:213-244: (kept trajectory indices in batch order, number of kept prompts)."""
    if metric_name == "seq_final_reward":
        vals = batch.batch["token_level_rewards"].sum(dim=-1).cpu().numpy()
    elif metric_name == "seq_reward":
        vals = batch.batch["token_level_scores"].sum(dim=-1).cpu().numpy()
    else:
        vals = np.asarray(batch.non_tensor_batch[metric_name])
    uid2vals = defaultdict(list)
    for uid, v in zip(batch.non_tensor_batch["uid"], vals, strict=True):
        uid2vals[uid].append(v)
    kept = {uid for uid, v in uid2vals.items() if np.std(v) > 0 or len(v) == 1}
    kept_idx = [i for i, uid in enumerate(batch.non_tensor_batch["uid"]) if uid in kept]
    return kept_idx, len(kept)


class RayDAPOTrainer(RayPPOTrainer):
    def __init__(self, config, reward_fn=None, train_dataloader=None, **kw):
        if reward_fn is None:
            rm = config.reward_model
            reward_fn = DAPOSyntheticRewardManager(seed=config.data.get("seed", 1234),
                                                   max_resp_len=config.data.max_response_length,
                                                   overlong_buffer_cfg=rm.get("overlong_buffer"))
        super().__init__(config, reward_fn=reward_fn, train_dataloader=train_dataloader, **kw)

    def step(self, batch_dict: dict | None = None) -> dict:
        """One DAPO training step: generation batches until the filtered batch is full, then the PPO update."""
        cfg = self.config
        fg = cfg.algorithm.get("filter_groups") or {}
        metrics, timing_raw = {}, {}
        batch, num_prompt_in_batch, num_gen_batches = None, 0, 0
        with marked_timer("step", timing_raw):
            while True:
                src = batch_dict if (batch_dict is not None and num_gen_batches == 0) else self.train_dataloader.next()
                num_gen_batches += 1
                new_batch = self._rollout(src, timing_raw)
                with marked_timer("reward", timing_raw):
                    reward_tensor, extra = compute_reward(new_batch, self.reward_fn)
                    new_batch.batch["token_level_scores"] = reward_tensor
                    if extra:
                        new_batch.non_tensor_batch.update({k: np.asarray(v) for k, v in extra.items()})
                    if cfg.algorithm.use_kl_in_reward:
                        # the recipe applies the penalty here, before any old log-prob exists (a TODO upstream)
                        raise NotImplementedError("use_kl_in_reward with the DAPO recipe")
                    new_batch.batch["token_level_rewards"] = new_batch.batch["token_level_scores"]
                if not fg.get("enable", False):
                    batch = new_batch
                    break
                kept_idx, n_kept = filter_groups(new_batch, fg.get("metric", "acc"))
                num_prompt_in_batch += n_kept
                new_batch = new_batch[kept_idx]
                batch = new_batch if batch is None else DataProto.concat([batch, new_batch])
                prompt_bsz = cfg.data.train_batch_size
                if num_prompt_in_batch < prompt_bsz:
                    max_num_gen_batches = fg.get("max_num_gen_batches", 0)
                    if max_num_gen_batches <= 0 or num_gen_batches < max_num_gen_batches:
                        continue
                    raise ValueError(f"{num_gen_batches=} >= {max_num_gen_batches=}. Generated too many. Please check "
                                     "if your data are too difficult. You could also try set max_num_gen_batches=0 "
                                     "to enable endless trials.")
                traj_bsz = prompt_bsz * cfg.actor_rollout_ref.rollout.n
                batch = batch[:traj_bsz]
                break
            batch = self._train_on(batch, metrics, timing_raw)
        metrics["train/num_gen_batches"] = num_gen_batches
        return self._finish_metrics(batch, metrics, timing_raw)

    def fit(self, num_steps=None):
        total = num_steps or self.config.trainer.get("total_training_steps") or 1
        self.global_steps = 1
        history = []
        for _ in range(total):
            history.append(self.step())
            self.global_steps += 1
        return history


def dapo_overrides(max_response_length: int, overlong_len: int | None = None):
    """The recipe's defaults (recipe/dapo/*.sh, config/dapo_trainer.yaml) as hydra-style overrides."""
    ob = overlong_len if overlong_len is not None else max(1, max_response_length // 4)
    return [
        "actor_rollout_ref.actor.clip_ratio_low=0.2", "actor_rollout_ref.actor.clip_ratio_high=0.28",
        "actor_rollout_ref.actor.clip_ratio_c=10.0", "actor_rollout_ref.actor.loss_agg_mode=token-mean",
        "actor_rollout_ref.actor.use_kl_loss=False", "actor_rollout_ref.actor.kl_loss_coef=0.0",
        "algorithm.use_kl_in_reward=False", "algorithm.adv_estimator=grpo",
        "+algorithm.filter_groups.enable=True", "+algorithm.filter_groups.metric=acc",
        "+algorithm.filter_groups.max_num_gen_batches=10",
        "+reward_model.overlong_buffer.enable=True", f"+reward_model.overlong_buffer.len={ob}",
        "+reward_model.overlong_buffer.penalty_factor=1.0", "+reward_model.overlong_buffer.log=False",
    ]


__all__ = ["RayDAPOTrainer", "filter_groups", "dapo_overrides"]
