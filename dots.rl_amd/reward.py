"""Reward managers (mirror of verl/workers/reward_manager/: registry.py, naive.py:27-122, dapo.py).

Every manager writes each response's score at its last valid response token (naive.py:100); the rest of
the (B, R) ``token_level_scores`` is zero.

* ``NaiveRewardManager`` ("naive"): the reference's rule-reward path — decode prompt and response with the
  tokenizer, score with ``compute_score`` (default: ``reward_score.default_compute_score``, gsm8k), or return
  ``rm_scores`` when a reward model already scored the batch (naive.py:55-60).
* ``SyntheticBernoulliRewardManager`` ("synthetic_bernoulli"): the benchmark reward of BASELINE.md §3
  (Bernoulli(0.5) per sequence, seeded) — no tokenizer or dataset exists offline.
* ``DAPOSyntheticRewardManager`` ("dapo_synthetic"): dapo.py's overlong-buffer penalty on the synthetic score.
"""

from __future__ import annotations

from collections import defaultdict

import numpy as np
import torch

from .protocol import DataProto
from .reward_score import default_compute_score

REWARD_MANAGER_REGISTRY: dict = {}


def register(name: str):
    """registry.py:24-41."""

    def decorator(cls):
        if name in REWARD_MANAGER_REGISTRY and REWARD_MANAGER_REGISTRY[name] != cls:
            raise ValueError(f"Reward manager {name} has already been registered: {REWARD_MANAGER_REGISTRY[name]} vs {cls}")
        REWARD_MANAGER_REGISTRY[name] = cls
        return cls

    return decorator


def get_reward_manager_cls(name: str):
    """registry.py:44-55."""
    if name not in REWARD_MANAGER_REGISTRY:
        raise ValueError(f"Unknown reward manager: {name}")
    return REWARD_MANAGER_REGISTRY[name]


@register("naive")
class NaiveRewardManager:
    """naive.py:27-122. The per-sample decode + score loop runs on the host (as in the reference); the batch
    tensors it reads are copied device->host once per call, and the reward tensor is returned on the
    responses' device."""

    def __init__(self, tokenizer, num_examine, compute_score=None, reward_fn_key="data_source"):
        self.tokenizer = tokenizer
        self.num_examine = num_examine
        self.compute_score = compute_score or default_compute_score
        self.reward_fn_key = reward_fn_key

    def __call__(self, data: DataProto, return_dict: bool = False):
        if "rm_scores" in data.batch.keys():  # naive.py:55-60
            if return_dict:
                return {"reward_tensor": data.batch["rm_scores"]}
            return data.batch["rm_scores"]
        responses = data.batch["responses"]
        B, R = responses.shape
        prompts = data.batch["prompts"].cpu().numpy()
        P = prompts.shape[-1]
        resp = responses.cpu().numpy()
        am = data.batch["attention_mask"].cpu().numpy()
        rewards = np.zeros(B, dtype=np.float32)
        last = np.zeros(B, dtype=np.int64)
        extra_out = defaultdict(list)
        printed = {}
        nt = data.non_tensor_batch
        for i in range(B):
            vpl = int(am[i, :P].sum())
            valid_prompt_ids = prompts[i, -vpl:]  # a zero-length prompt keeps the whole row (python's [-0:])
            vrl = int(am[i, P:].sum())
            valid_response_ids = resp[i, :vrl]
            prompt_str = self.tokenizer.decode(valid_prompt_ids, skip_special_tokens=True)
            response_str = self.tokenizer.decode(valid_response_ids, skip_special_tokens=True)
            ground_truth = nt["reward_model"][i]["ground_truth"]
            data_source = nt[self.reward_fn_key][i]
            extra_info = nt["extra_info"][i] if "extra_info" in nt else {}
            extra_info["num_turns"] = nt["__num_turns__"][i] if "__num_turns__" in nt else None
            score = self.compute_score(data_source=data_source, solution_str=response_str, ground_truth=ground_truth,
                                       extra_info=extra_info)
            if isinstance(score, dict):
                reward = score["score"]
                for k, v in score.items():
                    extra_out[k].append(v)
            else:
                reward = score
            rewards[i] = reward
            last[i] = vrl - 1 if vrl > 0 else R - 1  # reward_tensor[i, -1] for an empty response, as python indexes
            if printed.get(data_source, 0) < self.num_examine:
                printed[data_source] = printed.get(data_source, 0) + 1
                print("[prompt]", prompt_str)
                print("[response]", response_str)
                print("[ground_truth]", ground_truth)
                for k, v in (score.items() if isinstance(score, dict) else [("score", score)]):
                    print(f"[{k}]", v)
        out = torch.zeros(B, R, dtype=torch.float32)
        out[torch.arange(B), torch.from_numpy(last)] = torch.from_numpy(rewards)
        out = out.to(responses.device)
        if return_dict:
            return {"reward_tensor": out, "reward_extra_info": extra_out}
        return out


@register("synthetic_bernoulli")
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


@register("dapo_synthetic")
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


def load_reward_manager(config, tokenizer=None, num_examine: int = 0, compute_score=None, **reward_kwargs):
    """trainer/ppo/reward.py:93-148: the manager named by ``reward_model.reward_manager``. "naive" needs a
    tokenizer (decode) and scores with ``compute_score`` or default_compute_score; the synthetic managers take
    the data seed."""
    name = config.reward_model.get("reward_manager", "naive")
    cls = get_reward_manager_cls(name)
    if name == "naive":
        if tokenizer is None:
            raise ValueError("reward_manager=naive decodes responses: pass the tokenizer")
        return cls(tokenizer=tokenizer, num_examine=num_examine, compute_score=compute_score,
                   reward_fn_key=config.data.get("reward_fn_key", "data_source"), **reward_kwargs)
    return cls(seed=config.data.get("seed", 1234), **reward_kwargs)


def compute_reward(data: DataProto, reward_fn):
    """trainer/ppo/reward.py:151 — (reward_tensor, reward_extra_infos_dict)."""
    res = reward_fn(data, return_dict=True)
    return res["reward_tensor"], res.get("reward_extra_info", {})
