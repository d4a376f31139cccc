"""Trainer configuration with the reference's dotted key names (verl/trainer/config/ppo_trainer.yaml,
actor/actor.yaml, actor/dp_actor.yaml, rollout/rollout.yaml, algorithm section).

Only the keys the actor-learner hot path reads are defined; ``apply_overrides`` accepts the same
``a.b.c=value`` strings a hydra command line uses (e.g. ``actor_rollout_ref.actor.ppo_mini_batch_size=32``),
so reference launch scripts map over key for key. ``actor.strategy`` selects this backend: ``"mi355x"``.
"""

from __future__ import annotations

import ast
import copy


class AttrDict(dict):
    """dict with attribute access and ``.get`` — the subset of OmegaConf DictConfig in use."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    def __deepcopy__(self, memo):
        return AttrDict({k: copy.deepcopy(v, memo) for k, v in self.items()})


def to_attr(d):
    if isinstance(d, dict):
        return AttrDict({k: to_attr(v) for k, v in d.items()})
    if isinstance(d, list):
        return [to_attr(v) for v in d]
    return d


# Qwen2.5-0.5B architecture (config.json of Qwen/Qwen2.5-0.5B(-Instruct)); weights are random-init (no network)
QWEN25_05B = dict(
    vocab_size=151936, hidden_size=896, intermediate_size=4864, num_hidden_layers=24, num_attention_heads=14,
    num_key_value_heads=2, max_position_embeddings=32768, rope_theta=1000000.0, rms_norm_eps=1e-6,
    tie_word_embeddings=True, bos_token_id=151643, eos_token_id=151645, pad_token_id=151643,
)

# config #4 / #5 architectures (config.json of meta-llama/Meta-Llama-3-8B and Qwen/Qwen2.5-7B), random init
LLAMA3_8B = dict(
    vocab_size=128256, hidden_size=4096, intermediate_size=14336, num_hidden_layers=32, num_attention_heads=32,
    num_key_value_heads=8, max_position_embeddings=8192, rope_theta=500000.0, rms_norm_eps=1e-5,
    tie_word_embeddings=False, attention_bias=False, bos_token_id=128000, eos_token_id=128001, pad_token_id=128001,
    model_type="llama",
)
QWEN25_7B = dict(
    vocab_size=152064, hidden_size=3584, intermediate_size=18944, num_hidden_layers=28, num_attention_heads=28,
    num_key_value_heads=4, max_position_embeddings=32768, rope_theta=1000000.0, rms_norm_eps=1e-6,
    tie_word_embeddings=False, bos_token_id=151643, eos_token_id=151643, pad_token_id=151643,
)
RANDOM_MODELS = {"qwen2.5-0.5b": QWEN25_05B, "llama-3-8b": LLAMA3_8B, "qwen2.5-7b": QWEN25_7B}

# worker profiler (actor.yaml:133-160, critic.yaml, ProfilerConfig): tool "roctx" (rocprofv3 --marker-trace ranges) or
# "torch" (torch.profiler Chrome trace); which steps run between start_profile / stop_profile: global_profiler.steps
PROFILER = dict(tool=None, enable=False, all_ranks=False, ranks=[], save_path="outputs/profile")

DEFAULTS = dict(
    data=dict(train_batch_size=64, max_prompt_length=512, max_response_length=256, seed=1234,
              reward_fn_key="data_source"),
    actor_rollout_ref=dict(
        hybrid_engine=True,
        # share_prompt_prefix: the n samples of a prompt run its tokens once in the log-prob / update passes
        # (qwen2.PrefixShare: the per-token work of the prompt done once per group). Equal to the per-row passes in
        # fp32 up to summation order; in bf16 up to bf16 rounding (the copies' prompt gradients are summed in fp32 and
        # rounded once, and the GEMMs see other row counts), not bit-comparable — False restores per-row passes
        model=dict(path="random:qwen2.5-0.5b", override_config={}, use_remove_padding=False, use_fused_kernels=False,
                   share_prompt_prefix=True,
                   enable_gradient_checkpointing=False, external_lib=None, dtype="bfloat16"),
        actor=dict(
            strategy="mi355x", ppo_mini_batch_size=32, ppo_micro_batch_size=None, ppo_micro_batch_size_per_gpu=8,
            use_dynamic_bsz=False, ppo_max_token_len_per_gpu=16384, clip_ratio=0.2, clip_ratio_low=0.2,
            clip_ratio_high=0.2, clip_ratio_c=3.0, policy_loss=dict(loss_mode="vanilla"), loss_agg_mode="token-mean",
            entropy_coeff=0.0, use_kl_loss=True, kl_loss_coef=0.001, kl_loss_type="low_var_kl", ppo_epochs=1,
            shuffle=False, grad_clip=1.0, ulysses_sequence_parallel_size=1,
            # dp_actor.yaml:30-33: chunked / recomputed entropy bound the reference's (N, V) logits temporaries; K2
            # computes the entropy in the same single pass over the logits as the log-prob and keeps no temporaries,
            # so both are accepted and change nothing (dp_actor.DataParallelPPOActor)
            entropy_from_logits_with_chunking=False, entropy_checkpointing=False,
            # micro-batches run through the model together (one forward / backward over their concatenated rows; the
            # loss, its scale and the metrics stay per micro-batch): 0 = as many as fit exec_activation_gb of saved
            # activations, 1 = the reference's one micro-batch per pass (dp_actor.DataParallelPPOActor.update_policy)
            exec_micro_batches=0, exec_activation_gb=110,
            exec_log_prob_tokens=196608,  # forward-only log-prob passes: micro-batches per pass up to this many tokens
            # shard: fp32 master + AdamW moments split over the DP ranks (ZeRO-style; FSDP FULL_SHARD in the
            # reference); "auto" = when replicated state would exceed 64 GB per GPU (workers._shard_spec)
            fsdp_config=dict(shard="auto", fsdp_size=-1, param_offload=False, optimizer_offload=False),
            optim=dict(lr=1e-6, lr_warmup_steps_ratio=0.0, total_training_steps=-1, weight_decay=0.01,
                       lr_warmup_steps=-1, betas=[0.9, 0.999], eps=1e-8, warmup_style="constant", min_lr_ratio=0.0,
                       num_cycles=0.5),
            profiler=dict(PROFILER),
        ),
        rollout=dict(
            name="mi355x", mode="sync", temperature=1.0, top_k=-1, top_p=1.0, do_sample=True, n=8,
            prompt_length=512, response_length=256, ignore_eos=False, log_prob_micro_batch_size=None,
            log_prob_micro_batch_size_per_gpu=16, log_prob_use_dynamic_bsz=False, micro_batch_size=None,
            log_prob_max_token_len_per_gpu=16384,
            seed=1234, val_kwargs=dict(top_k=-1, top_p=1.0, temperature=0, n=1, do_sample=False),
            use_hip_graph=True,  # decode steps replayed from one captured HIP graph (rollout.py)
            packed_decode=True, packed_decode_max_rows=512,  # qwen2.PackedDecode (fragment-packed operands)
            decode_lm_head=True,  # PackedDecode's lm_head kernel at <= 64 rows (csrc/decode_gemm.hip)
            decode_fused_norm=False,  # PackedDecode's five-launch layer (norms in the consumer GEMMs): measured slower
            fused_select=False,  # lm_head fused with K4 (csrc/fused_linear.hip)
            decode_lanes=1,  # row groups of the graphed decode step on concurrent streams (rollout._decode_lanes)
            # rollout.yaml:177: emit `rollout_log_probs` (log p of each sampled token under the decode step's own
            # logits, -1 past the response) -> training/rollout_probs_diff_* metrics (ray_trainer.py:1221-1225)
            calculate_log_probs=False,
            # prefix caching of the n samples' shared prompt (vllm_rollout_spmd.py:195 runs vLLM with it on): each
            # distinct prompt prefilled once, its keys read from one cache row by the group's decode attention
            enable_prefix_caching=True,
            profiler=dict(PROFILER),
        ),
        ref=dict(log_prob_micro_batch_size=None, log_prob_micro_batch_size_per_gpu=16, log_prob_use_dynamic_bsz=False,
                 log_prob_max_token_len_per_gpu=16384, exec_log_prob_tokens=196608,
                 entropy_from_logits_with_chunking=False, entropy_checkpointing=False,  # dp_ref.yaml:43-46
                 profiler=dict(PROFILER)),
    ),
    # critic.yaml + dp_critic.yaml (used when algorithm.adv_estimator == "gae" or critic.enable)
    critic=dict(
        # None = the reference's ${oc.select:actor_rollout_ref...} interpolation (resolve_critic_config)
        strategy="mi355x", enable=None, rollout_n=None,
        fsdp_config=dict(shard="auto", fsdp_size=-1, param_offload=False, optimizer_offload=False),
        optim=dict(lr=1e-5, lr_warmup_steps_ratio=0.0, total_training_steps=-1, weight_decay=0.01, lr_warmup_steps=-1,
                   betas=[0.9, 0.999], eps=1e-8, warmup_style="constant", min_lr_ratio=0.0, num_cycles=0.5),
        model=dict(path="random:qwen2.5-0.5b", override_config={}, use_remove_padding=False, share_prompt_prefix=True,
                   dtype="bfloat16", seed=4321),
        ppo_mini_batch_size=None, ppo_micro_batch_size=None, ppo_micro_batch_size_per_gpu=8,
        forward_micro_batch_size=None, forward_micro_batch_size_per_gpu=16, use_dynamic_bsz=None,
        ppo_max_token_len_per_gpu=32768, forward_max_token_len_per_gpu=32768, ppo_epochs=None, shuffle=None,
        grad_clip=1.0, cliprange_value=0.5, loss_agg_mode=None, ulysses_sequence_parallel_size=1,
        exec_micro_batches=0, exec_activation_gb=110,  # as the actor's (dp_actor.exec_groups)
        profiler=dict(PROFILER),
    ),
    algorithm=dict(gamma=1.0, lam=1.0, adv_estimator="grpo", norm_adv_by_std_in_grpo=True, use_kl_in_reward=False,
                   kl_penalty="kl", kl_ctrl=dict(type="fixed", kl_coef=0.001, horizon=10000, target_kl=0.1)),
    reward_model=dict(enable=False, reward_manager="synthetic_bernoulli", launch_reward_fn_async=False),
    # ppo_trainer.yaml:269-290: the steps profiled (start_profile before, stop_profile after; ray_trainer.py:1096-1366)
    global_profiler=dict(tool=None, steps=None, profile_continuous_steps=False, save_path="outputs/profile"),
    # trainer.gc_freeze: freeze the host heap after init (trainer.freeze_host_heap; bench.py after its warmup)
    trainer=dict(balance_batch=False, gc_freeze=False, total_epochs=1, total_training_steps=None, critic_warmup=0, n_gpus_per_node=1,
                 nnodes=1, save_freq=-1, test_freq=-1, logger=["console"], project_name="dots_rl_amd",
                 experiment_name="grpo"),
)


def resolve_critic_config(cfg: AttrDict) -> AttrDict:
    """critic.yaml's interpolations from the actor (rollout_n, ppo_mini_batch_size, use_dynamic_bsz, ppo_epochs,
    shuffle, loss_agg_mode) for entries left None; returns cfg.critic."""
    c, a = cfg.critic, cfg.actor_rollout_ref.actor
    src = {"rollout_n": cfg.actor_rollout_ref.rollout.n, "ppo_mini_batch_size": a.ppo_mini_batch_size,
           "use_dynamic_bsz": a.use_dynamic_bsz, "ppo_epochs": a.ppo_epochs, "shuffle": a.shuffle,
           "loss_agg_mode": a.loss_agg_mode}
    for k, v in src.items():
        if c.get(k) is None:
            c[k] = v
    return c


def default_config():
    return to_attr(copy.deepcopy(DEFAULTS))


def _parse_value(s: str):
    low = s.lower()
    if low in ("true", "false"):
        return low == "true"
    if low in ("null", "none", "~"):
        return None
    try:
        return ast.literal_eval(s)
    except (ValueError, SyntaxError):
        return s


def apply_overrides(cfg: AttrDict, overrides) -> AttrDict:
    """Apply hydra-style ``a.b.c=value`` overrides in place (``+a.b=v`` adds a new key)."""
    for ov in overrides or []:
        key, _, val = ov.partition("=")
        add = key.startswith("+")
        key = key.lstrip("+")
        node = cfg
        parts = key.split(".")
        for p in parts[:-1]:
            if p not in node:
                if not add:
                    raise KeyError(f"unknown config key {key}")
                node[p] = AttrDict()
            node = node[p]
        if parts[-1] not in node and not add:
            raise KeyError(f"unknown config key {key}")
        node[parts[-1]] = to_attr(_parse_value(val))
    return cfg
