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

    def _scores(self, data: DataProto):
        responses = data.batch["responses"]
        g = torch.Generator(device=responses.device).manual_seed(self.seed + self.calls)
        self.calls += 1
        return torch.bernoulli(torch.full((responses.shape[0],), self.p, device=responses.device), generator=g)

    @staticmethod
    def _place(data: DataProto, reward):
        """reward_tensor[i, valid_response_length - 1] = reward[i] (naive.py:100; a length of 0 indexes -1, the
        last position, exactly as the reference's python indexing does)."""
        responses = data.batch["responses"]
        B, R = responses.shape
        valid_len = data.batch["attention_mask"][:, -R:].sum(-1)
        idx = torch.where(valid_len > 0, valid_len - 1, torch.full_like(valid_len, R - 1))
        out = torch.zeros(B, R, dtype=torch.float32, device=responses.device)
        out[torch.arange(B, device=responses.device), idx] = reward.to(torch.float32)
        return out, valid_len

    def __call__(self, data: DataProto, return_dict: bool = False):
        scores, _ = self._place(data, self._scores(data))
        if return_dict:
            return {"reward_tensor": scores, "reward_extra_info": {}}
        return scores


class DAPOSyntheticRewardManager(SyntheticBernoulliRewardManager):
    """reward_manager/dapo.py:26-150 with the synthetic score: reward = score + the overlong-buffer penalty
    min(-(L - (max_resp_len - buffer_len)) / buffer_len * penalty_factor, 0) (dapo.py:114-123), placed at the
    last valid response token; extra info `acc` (the score), `overlong_reward`, `overlong` when logging."""

    def __init__(self, seed: int = 1234, p: float = 0.5, max_resp_len=None, overlong_buffer_cfg=None):
        super().__init__(seed, p)
        self.overlong_buffer_cfg = overlong_buffer_cfg
        self.max_resp_len = max_resp_len
        if overlong_buffer_cfg is not None and overlong_buffer_cfg.get("enable", False):
            assert max_resp_len is not None, (
                f"max_resp_len must be provided if {overlong_buffer_cfg=}, but got None")
            assert max_resp_len >= overlong_buffer_cfg.len, "max_resp_len must be larger than overlong_buffer.len"

    def __call__(self, data: DataProto, return_dict: bool = False):
        score = self._scores(data)
        R = data.batch["responses"].shape[1]
        valid_len = data.batch["attention_mask"][:, -R:].sum(-1)
        reward = score.to(torch.float32)
        extra = {"acc": score.cpu().numpy()}
        ob = self.overlong_buffer_cfg
        if ob is not None and ob.get("enable", False):
            expected_len = self.max_resp_len - ob.len
            exceed_len = valid_len - expected_len
            overlong_reward = torch.clamp(-exceed_len / ob.len * ob.penalty_factor, max=0.0)
            reward = reward + overlong_reward
            if ob.get("log", False):
                extra["overlong_reward"] = overlong_reward.cpu().numpy()
                extra["overlong"] = (overlong_reward < 0).cpu().numpy()
        out, _ = self._place(data, reward)
        if return_dict:
            return {"reward_tensor": out, "reward_extra_info": extra}
        return out


def compute_reward(data: DataProto, reward_fn):
    """trainer/ppo/reward.py:151 — (reward_tensor, reward_extra_infos_dict)."""
    res = reward_fn(data, return_dict=True)
    return res["reward_tensor"], res.get("reward_extra_info", {})
