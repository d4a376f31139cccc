"""Child process of tests/test_dp_gpu.py (one DP rank; started by the test with subprocess, gloo backend,
both ranks on cuda:0). Runs ActorRolloutRefWorker.update_actor through the SPMD worker group - the
DP_COMPUTE_PROTO dispatch hands rank r the r-th chunk of the batch, FlatAdamW all-reduces (AVG) the flat
gradient - on the tiny Qwen2 in fp32 and saves the post-step parameters, metrics and grad norms."""

import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def build_config(world, shard=False):
    from dots.rl_amd.config import apply_overrides, default_config

    return apply_overrides(default_config(), [
        f"actor_rollout_ref.actor.fsdp_config.shard={'true' if shard else 'false'}",
        "actor_rollout_ref.rollout.n=1", "actor_rollout_ref.actor.ppo_mini_batch_size=4",
        "actor_rollout_ref.actor.ppo_micro_batch_size_per_gpu=1", "actor_rollout_ref.actor.optim.lr=1e-4",
        f"actor_rollout_ref.model.path={os.path.join(HERE, 'golden', 'tiny_qwen2')}",
        "actor_rollout_ref.model.dtype=float32",
    ]).actor_rollout_ref


def batch(device):
    from dots.rl_amd.protocol import DataProto

    z = np.load(os.path.join(HERE, "golden", "actor_update.npz"), allow_pickle=False)
    keys = ("input_ids", "attention_mask", "position_ids", "responses", "response_mask", "old_log_probs",
            "advantages", "ref_log_prob")
    return DataProto.from_dict({k: torch.from_numpy(z[f"c0_{k}"]).to(device) for k in keys},
                               meta_info={"temperature": 1.0})


def main(out_path, shard=False):
    import torch.distributed as dist

    from dots.rl_amd.single_controller import SPMDWorkerGroup, init_process_group_from_env
    from dots.rl_amd.workers import ActorRolloutRefWorker

    torch.cuda.set_device(0)
    init_process_group_from_env("gloo")
    world, rank = dist.get_world_size(), dist.get_rank()
    wg = SPMDWorkerGroup(ActorRolloutRefWorker(build_config(world, shard), role="actor"))
    wg.init_model()
    w = wg.worker
    out = wg.update_actor(batch("cuda"))
    torch.cuda.synchronize()
    st = w.store
    # full fp32 parameters in flat layout order: the small region + the (all-gathered) GEMM region
    params = torch.cat([st.small, st.compute[st.n_small:].float()]).cpu() if st.sharded else st.master.cpu()
    torch.save({"master": params, "sharded": st.sharded, "metrics": json.dumps(out.meta_info["metrics"]),
                "mini_batch_size": w.config.actor.ppo_mini_batch_size, "rank": rank, "world": world},
               out_path)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], shard=len(sys.argv) > 2 and sys.argv[2] == "shard")
