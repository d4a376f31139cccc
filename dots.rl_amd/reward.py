"""Reward managers (mirror of verl/workers/reward_manager/naive.py:46-122 placement semantics).

The score of each response is written at its last valid response token (naive.py:100); the rest of the
(B, R) ``token_level_scores`` is zero. ``SyntheticBernoulliRewardManager`` is the benchmark reward of
BASELINE.md §3 (Bernoulli(0.5) per sequence, seeded) — a rule reward needs a tokenizer and a dataset,
neither of which exists offline here.
"""

from __future__ import annotations

import torch

from .protocol import DataProto


class SyntheticBernoulliRewardManager:
    def __init__(self, seed: int = 1234, p: float = 0.5):
        self.seed = seed
        self.p = p
        self.calls = 0

    def __call__(self, data: DataProto, return_dict: bool = False):
        responses = data.batch["responses"]
        mask = data.batch["attention_mask"][:, -responses.shape[1]:]
        B, R = responses.shape
        g = torch.Generator(device=responses.device).manual_seed(self.seed + self.calls)
        self.calls += 1
        score = torch.bernoulli(torch.full((B,), self.p, device=responses.device), generator=g)
        valid_len = mask.sum(-1)
        scores = torch.zeros(B, R, dtype=torch.float32, device=responses.device)
        idx = (valid_len - 1).clamp(min=0)
        scores[torch.arange(B, device=responses.device), idx] = score
        if return_dict:
            return {"reward_tensor": scores, "reward_extra_info": {}}
        return scores


def compute_reward(data: DataProto, reward_fn):
    """trainer/ppo/reward.py:151 — (reward_tensor, reward_extra_infos_dict)."""
    res = reward_fn(data, return_dict=True)
    return res["reward_tensor"], res.get("reward_extra_info", {})
