"""PPO steps/sec + rollout tokens/sec for Qwen2.5-0.5B GRPO on MI355X (BASELINE.json config #2 / #3).

One "step" is one full GRPO iteration of RayPPOTrainer.fit(): rollout of 64 prompts x n=8 (512-token
prompts, 256-token responses, sampling) -> old log-probs + entropy -> ref log-probs -> GRPO advantages ->
two PPO mini-batch updates (micro 8/GPU) with AdamW. Global batch is fixed (512 sequences/step) and split
across the N ranks: "scaling" is strong. Random-init Qwen2.5-0.5B weights, synthetic prompts.

  python bench.py [--gpus N] [--steps K] [--warmup W]          (N>1 under torch.distributed.run)
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "PPO steps/sec + rollout tokens/sec, Qwen2.5-0.5B GRPO @1/2/4/8 MI355X"


def build_config(args):
    from dots.rl_amd.config import apply_overrides, default_config

    cfg = default_config()
    apply_overrides(cfg, [
        "data.train_batch_size=64", "data.max_prompt_length=512", "data.max_response_length=256",
        "actor_rollout_ref.rollout.n=8", "actor_rollout_ref.rollout.response_length=256",
        "actor_rollout_ref.rollout.prompt_length=512", "actor_rollout_ref.rollout.ignore_eos=True",
        "actor_rollout_ref.actor.ppo_mini_batch_size=32", "actor_rollout_ref.actor.ppo_micro_batch_size_per_gpu=8",
        "actor_rollout_ref.rollout.log_prob_micro_batch_size_per_gpu=16",
        "actor_rollout_ref.ref.log_prob_micro_batch_size_per_gpu=16",
        "actor_rollout_ref.actor.use_kl_loss=True", "actor_rollout_ref.actor.kl_loss_coef=0.001",
        "actor_rollout_ref.actor.kl_loss_type=low_var_kl", "actor_rollout_ref.actor.entropy_coeff=0",
        "algorithm.adv_estimator=grpo", "trainer.balance_batch=False",
    ])
    if args.tiny:
        apply_overrides(cfg, ["+actor_rollout_ref.model.override_config.num_hidden_layers=2",
                              "data.train_batch_size=8", "actor_rollout_ref.actor.ppo_mini_batch_size=4",
                              "actor_rollout_ref.actor.ppo_micro_batch_size_per_gpu=4",
                              "data.max_response_length=32", "actor_rollout_ref.rollout.response_length=32",
                              "data.max_prompt_length=64", "actor_rollout_ref.rollout.prompt_length=64"])
    apply_overrides(cfg, args.override)
    return cfg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--tiny", action="store_true", help="2-layer model, small batch (bring-up only)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--override", nargs="*", default=[])
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from dots.rl_amd.single_controller import init_process_group_from_env
    from dots.rl_amd.trainer import RayPPOTrainer

    init_process_group_from_env()
    rank, world = dist.get_rank(), dist.get_world_size()
    assert world == args.gpus, f"--gpus {args.gpus} but WORLD_SIZE {world}"
    cfg = build_config(args)
    trainer = RayPPOTrainer(cfg)
    trainer.init_workers()
    trainer.global_steps = 1
    for _ in range(args.warmup):
        trainer.step(trainer.train_dataloader.next())
        trainer.global_steps += 1
    prompts = [trainer.train_dataloader.next() for _ in range(args.steps)]
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    hist = []
    for p in prompts:
        hist.append(trainer.step(p))
        trainer.global_steps += 1
    torch.cuda.synchronize()
    dist.barrier()
    elapsed = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cuda")
    dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    elapsed = float(elapsed.item())
    steps_per_s = args.steps / elapsed
    gen_tokens = sum(h["perf/total_num_tokens"] for h in hist)  # prompt + response tokens processed
    resp_tokens = sum(h["perf/rollout_tokens_per_sec"] * h["timing_s/gen"] for h in hist)
    gen_time = sum(h["timing_s/gen"] for h in hist)
    if rank == 0:
        ar = cfg.actor_rollout_ref
        line = {
            "metric": METRIC,
            "value": steps_per_s,
            "unit": "PPO steps/s",
            "rollout_tokens_per_sec": resp_tokens / gen_time,
            "perf/throughput_tokens_per_sec_per_gpu": gen_tokens / elapsed / world,
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic",
            "config": {"workload": "Qwen2.5-0.5B GRPO, 64 prompts x n=8, 512-tok prompts / 256-tok responses",
                       "model": "Qwen2.5-0.5B (random init)", "global_batch": cfg.data.train_batch_size * ar.rollout.n,
                       "seq_len": cfg.data.max_prompt_length + cfg.data.max_response_length,
                       "parallelism": f"dp{world}", "tiny": bool(args.tiny)},
            "timing_s": {k.split("/", 1)[1]: sum(h[k] for h in hist) / len(hist) for k in hist[0] if k.startswith("timing_s/")},
            "mfu_actor": sum(h.get("perf/mfu/actor", 0.0) for h in hist) / len(hist),
        }
        print(json.dumps(line), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
