"""RayPPOTrainer.fit() dataflow on the SPMD single controller (mirror of verl/trainer/ppo/ray_trainer.py).

One PPO step (ray_trainer.py:1104-1399): prompts -> uid -> repeat(n, interleave) -> generate_sequences ->
union -> response_mask -> (balance_batch) -> global_token_num -> reward -> compute_log_prob (old log-probs
+ entropy) -> compute_ref_log_prob -> advantage (GRPO / GAE on device) -> update_actor -> metrics.
The "driver" runs on every rank (SPMD); worker-group calls dispatch this rank's DP chunk and all-gather
the outputs, so the full batch is resident in each rank's HBM between stages (no object-store hops).
"""

from __future__ import annotations

import gc
import os
import time
import uuid
from contextlib import contextmanager

import numpy as np
import torch
import torch.distributed as dist

from . import core_algos
from .core_algos import AdvantageEstimator, agg_loss
from .metric_utils import (calculate_debug_metrics, compute_data_metrics, compute_throughout_metrics,
                           compute_timing_metrics, reduce_metrics)
from .protocol import DataProto
from .reward import compute_reward, load_reward_manager
from .seqlen_balancing import get_seqlen_balanced_partitions, log_seqlen_unbalance
from .single_controller import SPMDWorkerGroup
from .config import resolve_critic_config
from .workers import ActorRolloutRefWorker, CriticWorker


_ALLOC_TRACE = os.environ.get("DRL_ALLOC_TRACE", "0") == "1"


@contextmanager
def marked_timer(name: str, timing_raw: dict):
    """profiler/performance.py:172 — wall time of a stage (synchronised: stages run on the GPU stream)."""
    sync = torch.cuda.is_initialized()  # host-only callers (CPU tests of the driver logic) have no stream
    if sync:
        torch.cuda.synchronize()
    trace = sync and _ALLOC_TRACE
    a0 = torch.cuda.memory_stats().get("num_device_alloc", 0) if trace else 0
    t0 = time.perf_counter()
    yield
    if sync:
        torch.cuda.synchronize()
    timing_raw[name] = timing_raw.get(name, 0.0) + time.perf_counter() - t0
    if trace:  # DRL_ALLOC_TRACE=1: device allocations of torch's caching allocator inside the stage
        key = name + "_device_allocs"
        timing_raw[key] = timing_raw.get(key, 0) + torch.cuda.memory_stats().get("num_device_alloc", 0) - a0


def compute_response_mask(data: DataProto):
    """ray_trainer.py:196-211."""
    R = data.batch["responses"].size(1)
    return data.batch["attention_mask"][:, -R:]


def apply_kl_penalty(data: DataProto, kl_ctrl, kl_penalty="kl"):
    """ray_trainer.py:154-193 (use_kl_in_reward)."""
    mask = data.batch["response_mask"]
    kld = core_algos.kl_penalty(data.batch["old_log_probs"], data.batch["ref_log_prob"], kl_penalty) * mask
    beta = kl_ctrl.value
    data.batch["token_level_rewards"] = data.batch["token_level_scores"] - beta * kld
    current_kl = float(core_algos.agg_loss(kld, mask, "token-mean"))
    kl_ctrl.update(current_kl=current_kl, n_steps=len(data))
    return data, {"actor/reward_kl_penalty": current_kl, "actor/reward_kl_penalty_coeff": beta}


def compute_advantage(data: DataProto, adv_estimator, gamma=1.0, lam=1.0, num_repeat=1, norm_adv_by_std_in_grpo=True,
                      config=None) -> DataProto:
    """ray_trainer.py:214-291."""
    if "response_mask" not in data.batch:
        data.batch["response_mask"] = compute_response_mask(data)
    if adv_estimator == AdvantageEstimator.GAE:
        adv, ret = core_algos.compute_gae_advantage_return(data.batch["token_level_rewards"], data.batch["values"],
                                                           data.batch["response_mask"], gamma, lam)
    elif adv_estimator == AdvantageEstimator.GRPO:
        adv, ret = core_algos.compute_grpo_outcome_advantage(
            token_level_rewards=data.batch["token_level_rewards"], response_mask=data.batch["response_mask"],
            index=data.non_tensor_batch["uid"], norm_adv_by_std_in_grpo=norm_adv_by_std_in_grpo)
    else:
        fn = core_algos.get_adv_estimator_fn(adv_estimator)
        kw = {"token_level_rewards": data.batch["token_level_rewards"], "response_mask": data.batch["response_mask"],
              "config": config}
        if "uid" in data.non_tensor_batch:
            kw["index"] = data.non_tensor_batch["uid"]
        if "reward_baselines" in data.batch:
            kw["reward_baselines"] = data.batch["reward_baselines"]
        adv, ret = fn(**kw)
    data.batch["advantages"] = adv
    data.batch["returns"] = ret
    return data


def freeze_host_heap():
    """trainer.gc_freeze (ours; for long-running jobs): move the long-lived host objects (workers, parameter views,
    configs, the warmed-up caches) to the collector's permanent generation. A full collection otherwise re-scans them —
    tens of ms of host time that lands wherever the allocation count trips it, and at a stage boundary (a
    synchronisation) the GPU waits it out: a 40 ms idle stretch at the start of a step in the kernel trace
    (profiles/r05_trace_summary_idle.txt). Objects frozen here are never collected as cycles, so call it once the
    process holds what it keeps (bench.py: after the warmup steps)."""
    gc.collect()
    gc.freeze()


class SyntheticPromptLoader:
    """Fixed-length synthetic prompts: token ids ~ U[0, vocab_limit), no padding (vocab_limit is
    also the pad id of left-padded rows, so it must be a valid embedding row)."""

    def __init__(self, batch_size, prompt_length, vocab_limit=151643, seed=1234, device="cuda", left_pad=None):
        self.batch_size = batch_size
        self.prompt_length = prompt_length
        self.vocab_limit = vocab_limit
        self.seed = seed
        self.device = device
        self.left_pad = left_pad  # optional (B,) number of left-pad tokens for variable-length prompts
        self.step = 0

    def next(self) -> dict:
        g = torch.Generator(device=self.device).manual_seed(self.seed + self.step)
        self.step += 1
        B, P = self.batch_size, self.prompt_length
        ids = torch.randint(0, self.vocab_limit, (B, P), generator=g, device=self.device)
        am = torch.ones(B, P, dtype=torch.int64, device=self.device)
        if self.left_pad is not None:
            for i, n in enumerate(self.left_pad):
                am[i, :n] = 0
                ids[i, :n] = self.vocab_limit  # pad id
        from .torch_functional import compute_position_id_with_mask

        pos = compute_position_id_with_mask(am)
        return {"input_ids": ids, "attention_mask": am, "position_ids": pos}


class RayPPOTrainer:
    """The fit() loop of ray_trainer.py:1050-1405 for the GRPO/PPO actor-learner hot path."""

    def __init__(self, config, reward_fn=None, train_dataloader=None, eos_token_id=None, pad_token_id=None,
                 tokenizer=None, rm_wg=None):
        self.config = config
        if eos_token_id is None or pad_token_id is None:
            # the model's own special ids (Qwen2.5: 151645 / 151643; Llama-3-8B: 128001 / 128001), as the
            # reference takes them from the tokenizer / generation config of the loaded model
            from .workers import resolve_model_config

            mc = resolve_model_config(config.actor_rollout_ref.model)
            eos_token_id = mc.eos_token_id if eos_token_id is None else eos_token_id
            pad_token_id = mc.pad_token_id if pad_token_id is None else pad_token_id
        self.tokenizer = tokenizer
        self.reward_fn = reward_fn or load_reward_manager(config, tokenizer)
        # reward model scores (ray_trainer.py:1200-1203): a worker group with compute_rm_score(batch) -> DataProto
        # holding `rm_scores`; the reward model itself is outside this repository's path
        self.use_rm = bool(config.reward_model.get("enable", False))
        self.rm_wg = rm_wg
        if train_dataloader is None:
            # token ids below the model's vocabulary (Qwen2.5: its 151643 text tokens; Llama-3: 128256 rows)
            from .workers import resolve_model_config

            vocab = resolve_model_config(config.actor_rollout_ref.model).vocab_size
            train_dataloader = SyntheticPromptLoader(config.data.train_batch_size, config.data.max_prompt_length,
                                                     vocab_limit=min(151643, vocab - 1),
                                                     seed=config.data.get("seed", 1234))
        self.train_dataloader = train_dataloader
        self.eos_token_id = eos_token_id
        self.pad_token_id = pad_token_id
        self.use_reference_policy = config.actor_rollout_ref.actor.use_kl_loss or config.algorithm.use_kl_in_reward
        self.kl_ctrl_in_reward = core_algos.get_kl_controller(config.algorithm.kl_ctrl)
        # ray_trainer.py:340-356: a critic when critic.enable says so, else exactly for GAE
        enable = config.get("critic", {}).get("enable") if "critic" in config else None
        if enable is not None:
            self.use_critic = bool(enable)
        else:
            self.use_critic = config.algorithm.adv_estimator == AdvantageEstimator.GAE.value
        self.global_steps = 0
        self.n_gpus = dist.get_world_size() if dist.is_initialized() else 1
        # ray_trainer.py:557-571: the schedule horizon of the actor / critic LR schedules — the dataloader's length x
        # total_epochs, unless trainer.total_training_steps overrides it (the synthetic loader is endless: no length)
        total = config.trainer.get("total_training_steps")
        if total is None and hasattr(train_dataloader, "__len__"):
            total = len(train_dataloader) * int(config.trainer.get("total_epochs", 1))
        self.total_training_steps = total
        if total is not None:
            config.actor_rollout_ref.actor.optim.total_training_steps = int(total)
            if "critic" in config:
                config.critic.optim.total_training_steps = int(total)

    def init_workers(self):
        """ray_trainer.py:779-886: one colocated actor/rollout/ref worker per GPU (hybrid engine)."""
        worker = ActorRolloutRefWorker(self.config.actor_rollout_ref, role="actor_rollout_ref")
        self.actor_rollout_wg = SPMDWorkerGroup(worker)
        self.ref_policy_wg = self.actor_rollout_wg
        if self.use_critic:
            self.critic_wg = SPMDWorkerGroup(CriticWorker(resolve_critic_config(self.config)))
            self.critic_wg.init_model()
        self.actor_rollout_wg.init_model()
        if self.config.trainer.get("gc_freeze", False):
            freeze_host_heap()

    def _uids(self, n):
        # deterministic and unique across generation batches (uuid4 in the reference; only group identity matters)
        base = getattr(self, "_uid_next", 0)
        self._uid_next = base + n
        return np.array([str(uuid.UUID(int=(self.global_steps << 40) + base + i)) for i in range(n)], dtype=object)

    def _balance_batch(self, batch: DataProto, metrics, logging_prefix="global_seqlen"):
        """ray_trainer.py:1033-1048: reorder rows so every DP rank's contiguous chunk carries a similar token
        count (Karmarkar-Karp, equal-size partitions)."""
        am = batch.batch["attention_mask"]
        seqlens = am.view(am.shape[0], -1).sum(-1).tolist()
        parts = None
        uid = batch.non_tensor_batch.get("uid")
        if self.config.actor_rollout_ref.model.get("share_prompt_prefix", True) and uid is not None:
            # prefix sharing runs a prompt's tokens once per rank that holds its samples: balance whole prompt
            # groups (same Karmarkar-Karp over the groups' token sums) so each group stays on one rank
            groups = {}
            for i, u in enumerate(uid.tolist()):
                groups.setdefault(u, []).append(i)
            rows = list(groups.values())
            if len({len(r) for r in rows}) == 1 and len(rows) % self.n_gpus == 0:
                gsum = [sum(seqlens[i] for i in r) for r in rows]
                gparts = get_seqlen_balanced_partitions(gsum, k_partitions=self.n_gpus, equal_size=True)
                parts = [[i for g in gp for i in rows[g]] for gp in gparts]
        if parts is None:
            parts = get_seqlen_balanced_partitions(seqlens, k_partitions=self.n_gpus, equal_size=True)
        batch.reorder(torch.tensor([j for p in parts for j in p], device=am.device))
        metrics.update(log_seqlen_unbalance(seqlens, parts, logging_prefix))

    def _rollout(self, batch_dict: dict, timing_raw: dict) -> DataProto:
        """ray_trainer.py:1104-1170: uid per prompt, repeat(n, interleave), generate_sequences, union."""
        ar = self.config.actor_rollout_ref
        batch = DataProto.from_single_dict(batch_dict)
        batch.non_tensor_batch["uid"] = self._uids(len(batch))
        gen_batch = batch.pop(batch_keys=["input_ids", "attention_mask", "position_ids"])
        gen_batch.meta_info.update({"global_steps": self.global_steps, "eos_token_id": self.eos_token_id,
                                    "pad_token_id": self.pad_token_id})
        base_batch = gen_batch
        gen_batch = gen_batch.repeat(repeat_times=ar.rollout.n, interleave=True)
        with marked_timer("gen", timing_raw):
            gen_out = self.actor_rollout_wg.generate_sequences(gen_batch)
            for k, v in gen_out.meta_info.pop("timing", {}).items():
                timing_raw[k] = timing_raw.get(k, 0.0) + v
        if str(getattr(self.config.algorithm.adv_estimator, "value", self.config.algorithm.adv_estimator)) == "remax":
            # ray_trainer.py:1160-1180: one greedy response per prompt, scored by the reward function; its sum is the
            # prompt's baseline, repeated with the batch below
            if self.reward_fn is None:
                raise ValueError("A reward_fn is required for REMAX advantage estimation.")
            with marked_timer("gen_max", timing_raw):
                base_batch.meta_info["do_sample"] = False
                base_out = self.actor_rollout_wg.generate_sequences(base_batch)
                base_out.meta_info.pop("timing", None)
                batch = batch.union(base_out)  # in place, as the reference's
                rb = self.reward_fn(batch)
                rb = rb["reward_tensor"] if isinstance(rb, dict) else rb
                batch.pop(batch_keys=list(base_out.batch.keys()))
                batch.batch["reward_baselines"] = rb.sum(dim=-1)
                del base_out
        batch = batch.repeat(repeat_times=ar.rollout.n, interleave=True)
        return batch.union(gen_out)

    def _train_on(self, batch: DataProto, metrics: dict, timing_raw: dict) -> DataProto:
        """ray_trainer.py:1171-1375: response mask, balance, reward (unless the caller already scored the batch),
        old log-prob + entropy, ref log-prob, values, advantage, update_critic, update_actor."""
        cfg = self.config
        ar = cfg.actor_rollout_ref
        if "response_mask" not in batch.batch:
            batch.batch["response_mask"] = compute_response_mask(batch)
        if cfg.trainer.balance_batch and self.n_gpus > 1:
            self._balance_batch(batch, metrics)
        batch.meta_info["global_token_num"] = batch.batch["attention_mask"].sum(-1).tolist()
        reward_tensor, reward_extra = None, {}
        if "token_level_scores" not in batch.batch:
            with marked_timer("reward", timing_raw):
                if self.use_rm:
                    if self.rm_wg is None:
                        raise NotImplementedError("reward_model.enable=True needs an rm_wg (compute_rm_score)")
                    batch = batch.union(self.rm_wg.compute_rm_score(batch))
                reward_tensor, reward_extra = compute_reward(batch, self.reward_fn)
        with marked_timer("old_log_prob", timing_raw):
            old = self.actor_rollout_wg.compute_log_prob(batch)
            ent = agg_loss(old.batch["entropys"], batch.batch["response_mask"], ar.actor.loss_agg_mode)
            metrics["actor/entropy"] = ent
            old.batch.pop("entropys")
            batch = batch.union(old)
            if "rollout_log_probs" in batch.batch:  # rollout.calculate_log_probs (ray_trainer.py:1221-1225)
                metrics.update(calculate_debug_metrics(batch))
        if self.use_reference_policy:
            with marked_timer("ref", timing_raw):
                batch = batch.union(self.ref_policy_wg.compute_ref_log_prob(batch))
        if self.use_critic:
            with marked_timer("values", timing_raw):
                batch = batch.union(self.critic_wg.compute_values(batch))
        with marked_timer("adv", timing_raw):
            if reward_tensor is not None:
                batch.batch["token_level_scores"] = reward_tensor
            if reward_extra:
                batch.non_tensor_batch.update({k: np.array(v) for k, v in reward_extra.items()})
            if "token_level_rewards" not in batch.batch:
                if cfg.algorithm.use_kl_in_reward:
                    batch, klm = apply_kl_penalty(batch, self.kl_ctrl_in_reward, cfg.algorithm.kl_penalty)
                    metrics.update(klm)
                else:
                    batch.batch["token_level_rewards"] = batch.batch["token_level_scores"]
            batch = compute_advantage(batch, cfg.algorithm.adv_estimator, cfg.algorithm.gamma, cfg.algorithm.lam,
                                      ar.rollout.n, cfg.algorithm.norm_adv_by_std_in_grpo, cfg.algorithm)
        if self.use_critic:
            with marked_timer("update_critic", timing_raw):
                critic_out = self.critic_wg.update_critic(batch)
            metrics.update(reduce_metrics(critic_out.meta_info["metrics"]))
        if cfg.trainer.critic_warmup <= self.global_steps:
            with marked_timer("update_actor", timing_raw):
                batch.meta_info["multi_turn"] = False
                batch.meta_info["temperature"] = ar.rollout.temperature
                actor_out = self.actor_rollout_wg.update_actor(batch)
            metrics.update(reduce_metrics(actor_out.meta_info["metrics"]))
        return batch

    def _finish_metrics(self, batch: DataProto, metrics: dict, timing_raw: dict) -> dict:
        """ray_trainer.py:1377-1399."""
        metrics["actor/entropy"] = float(metrics["actor/entropy"])
        metrics.update({"training/global_step": self.global_steps})
        metrics.update(compute_data_metrics(batch, use_critic=self.use_critic))
        metrics.update(compute_timing_metrics(batch, timing_raw))
        metrics.update(compute_throughout_metrics(batch, timing_raw, self.n_gpus))
        n_resp = batch.batch["response_mask"].sum().item()
        metrics["perf/rollout_tokens_per_sec"] = n_resp / timing_raw["gen"]
        self.last_batch = batch
        return metrics

    def step(self, batch_dict: dict) -> dict:
        """One PPO step — ray_trainer.py:1104-1399 minus validation/checkpoint/logging."""
        metrics, timing_raw = {}, {}
        with marked_timer("step", timing_raw):
            batch = self._rollout(batch_dict, timing_raw)
            batch = self._train_on(batch, metrics, timing_raw)
        return self._finish_metrics(batch, metrics, timing_raw)

    def _profile_wgs(self):
        wgs = [self.actor_rollout_wg]
        if self.use_reference_policy and self.ref_policy_wg is not self.actor_rollout_wg:
            wgs.append(self.ref_policy_wg)
        if self.use_critic:
            wgs.append(self.critic_wg)
        if self.use_rm and self.rm_wg is not None and hasattr(self.rm_wg, "start_profile"):
            wgs.append(self.rm_wg)
        return wgs

    def _start_profiling(self, do_profile: bool) -> None:
        """ray_trainer.py:1011-1020 (the ref worker is the actor's own colocated worker: started once)."""
        if do_profile:
            for i, wg in enumerate(self._profile_wgs()):
                if i == 0:
                    wg.start_profile(role="e2e", profile_step=self.global_steps)
                else:
                    wg.start_profile()

    def _stop_profiling(self, do_profile: bool) -> None:
        """ray_trainer.py:1022-1031."""
        if do_profile:
            for wg in self._profile_wgs():
                wg.stop_profile()

    def fit(self, num_steps=None):
        """ray_trainer.py:1050-1405 training loop (synthetic data; no validation/checkpoint by default), with the
        global_profiler step selection of :1096-1113 / :1355-1366."""
        total = num_steps or self.total_training_steps or 1
        gp = self.config.get("global_profiler", {}) or {}
        steps = gp.get("steps")
        continuous = bool(gp.get("profile_continuous_steps", False))
        self.global_steps = 1
        history = []
        prev_p, cur_p = False, (self.global_steps in steps) if steps is not None else False
        for _ in range(total):
            self._start_profiling((not prev_p and cur_p) if continuous else cur_p)
            m = self.step(self.train_dataloader.next())
            next_p = (self.global_steps + 1 in steps) if steps is not None else False
            self._stop_profiling((cur_p and not next_p) if continuous else cur_p)
            prev_p, cur_p = cur_p, next_p
            history.append(m)
            self.global_steps += 1
        return history
