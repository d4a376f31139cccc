"""trainer._balance_batch under prefix sharing: whole prompt groups (the n samples of a uid) are balanced over the DP
ranks with the reference's Karmarkar-Karp (ray_trainer.py:1033-1048 balances rows), so every rank's contiguous
chunk holds complete groups and the token sums stay balanced; with sharing off, the reference's row balancing."""
from types import SimpleNamespace

import numpy as np
import torch

from dots.rl_amd.config import apply_overrides, default_config
from dots.rl_amd.protocol import DataProto
from dots.rl_amd.trainer import RayPPOTrainer


def _batch(prompts, n, seed):
    g = torch.Generator().manual_seed(seed)
    B, T = prompts * n, 64
    am = torch.zeros(B, T, dtype=torch.int64)
    for b in range(B):
        am[b, : int(torch.randint(16, T + 1, (1,), generator=g))] = 1
    uid = np.array([f"u{b // n}" for b in range(B)], dtype=object)
    return DataProto.from_dict({"attention_mask": am, "row": torch.arange(B)}, {"uid": uid})


def test_group_balancing_keeps_groups_on_one_rank():
    cfg = default_config()
    world, n = 4, 8
    batch = _batch(16, n, 0)
    seqlens = batch.batch["attention_mask"].sum(-1)
    metrics = {}
    RayPPOTrainer._balance_batch(SimpleNamespace(n_gpus=world, config=cfg), batch, metrics)
    rows = batch.batch["row"]
    assert sorted(rows.tolist()) == list(range(16 * n))
    chunk = len(rows) // world
    sums = []
    for r in range(world):
        part = rows[r * chunk:(r + 1) * chunk].tolist()
        groups = {p // n for p in part}
        assert all(sum(1 for p in part if p // n == gi) == n for gi in groups)  # whole groups only
        sums.append(int(seqlens[part].sum()))
    assert max(sums) - min(sums) <= max(int(seqlens.view(-1, n).sum(-1).max()), 1)
    assert metrics["global_seqlen/balanced_max"] == max(sums)


def test_row_balancing_without_sharing():
    cfg = apply_overrides(default_config(), ["actor_rollout_ref.model.share_prompt_prefix=False"])
    batch = _batch(16, 8, 1)
    RayPPOTrainer._balance_batch(SimpleNamespace(n_gpus=4, config=cfg), batch, {})
    rows = batch.batch["row"].tolist()
    # the reference's row-level partitions split groups across ranks
    assert any(len({p // 8 for p in rows[r * 32:(r + 1) * 32]}) > 4 for r in range(4))
