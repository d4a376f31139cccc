"""Step metrics with the reference's keys (verl/trainer/ppo/metric_utils.py:80-302)."""

from __future__ import annotations

from typing import Any

import numpy as np
import torch

from .protocol import DataProto


def reduce_metrics(metrics: dict) -> dict:
    """metric_utils.py reduce_metrics: mean of each list."""
    return {k: float(np.mean(v)) if isinstance(v, (list, tuple)) else v for k, v in metrics.items()}


def _response_info(batch: DataProto):
    R = batch.batch["responses"].shape[-1]
    am = batch.batch["attention_mask"]
    return {"prompt_length": am[:, :-R].sum(-1).float(), "response_length": am[:, -R:].sum(-1).float(),
            "response_mask": am[:, -R:].bool()}


def compute_data_metrics(batch: DataProto, use_critic: bool = False) -> dict[str, Any]:
    """metric_utils.py:80-224: score / reward statistics over the non-aborted rows (response length > 0),
    advantages / returns (/ values) over the response mask, response and prompt length statistics. Every
    statistic is reduced on the device and read back in one copy."""
    b = batch.batch
    seq_score = b["token_level_scores"].sum(-1)
    seq_reward = b["token_level_rewards"].sum(-1)
    R = b["responses"].shape[-1]
    info = _response_info(batch)
    rmask = b["response_mask"].bool()
    resp_len, prompt_len = info["response_length"], info["prompt_length"]
    non_aborted = resp_len != 0
    if not bool(non_aborted.any()):
        raise ValueError("All samples are aborted, this should not happen.")
    sc, rw, rl = seq_score[non_aborted], seq_reward[non_aborted], resp_len[non_aborted]
    adv = torch.masked_select(b["advantages"], rmask)
    ret = torch.masked_select(b["returns"], rmask)
    P = b["attention_mask"].shape[-1] - R

    def mmm(x):
        return [x.mean(), x.max(), x.min()]

    vals = torch.stack([
        *mmm(sc), *mmm(rw), *mmm(adv.float()), *mmm(ret.float()),
        *mmm(resp_len), (resp_len == R).float().mean(),
        *mmm(rl), (rl == R).float().mean(), (~non_aborted).float().mean(),
        *mmm(prompt_len), (prompt_len == P).float().mean()]).cpu().tolist()
    keys = ["critic/score/mean", "critic/score/max", "critic/score/min", "critic/rewards/mean", "critic/rewards/max",
            "critic/rewards/min", "critic/advantages/mean", "critic/advantages/max", "critic/advantages/min",
            "critic/returns/mean", "critic/returns/max", "critic/returns/min", "response_length/mean",
            "response_length/max", "response_length/min", "response_length/clip_ratio",
            "response_length_non_aborted/mean", "response_length_non_aborted/max", "response_length_non_aborted/min",
            "response_length_non_aborted/clip_ratio", "response/aborted_ratio", "prompt_length/mean",
            "prompt_length/max", "prompt_length/min", "prompt_length/clip_ratio"]
    out = dict(zip(keys, vals))
    if use_critic:  # metric_utils.py:138-143, 176-186
        v = torch.masked_select(b["values"], rmask)
        rdv, rv = torch.var(ret - v), torch.var(ret)
        cv = torch.stack([v.mean(), v.max(), v.min(), 1.0 - rdv / (rv + 1e-5)]).float().cpu().tolist()
        out.update(dict(zip(["critic/values/mean", "critic/values/max", "critic/values/min",
                             "critic/vf_explained_var"], cv)))
    for k in ("__num_turns__", "tool_call_counts"):  # metric_utils.py:210-222
        if k in batch.non_tensor_batch:
            arr = batch.non_tensor_batch[k]
            name = "num_turns" if k == "__num_turns__" else k
            out.update({f"{name}/min": arr.min(), f"{name}/max": arr.max(), f"{name}/mean": arr.mean()})
    return out


def compute_timing_metrics(batch: DataProto, timing_raw: dict) -> dict[str, Any]:
    """metric_utils.py:227-266."""
    info = _response_info(batch)
    n_prompt = float(info["prompt_length"].sum().item())
    n_resp = float(info["response_length"].sum().item())
    n_all = n_prompt + n_resp
    sec = {"gen": n_resp, **{k: n_all for k in ["ref", "values", "adv", "update_critic", "update_actor"]}}
    return {**{f"timing_s/{k}": v for k, v in timing_raw.items()},
            **{f"timing_per_token_ms/{k}": timing_raw[k] * 1000 / sec[k] for k in set(sec) & set(timing_raw)}}


def compute_throughout_metrics(batch: DataProto, timing_raw: dict, n_gpus: int) -> dict[str, Any]:
    """metric_utils.py:269-302: perf/throughput = sum(attention-mask tokens) / (t_step * n_gpus)."""
    total = sum(batch.meta_info["global_token_num"])
    t = timing_raw["step"]
    return {"perf/total_num_tokens": total, "perf/time_per_step": t, "perf/throughput": total / (t * n_gpus)}


def calculate_debug_metrics(data: DataProto) -> dict:
    """utils/debug/metrics.py:63-108 (ray_trainer.py:1221-1225, when the rollout emitted ``rollout_log_probs``):
    rollout-vs-actor probabilities p = exp(log p) over the response mask (``response_mask``, else the response part
    of ``attention_mask``) — |p_actor - p_rollout| max / mean / std (unbiased) and their Pearson correlation."""
    b = data.batch
    rlp, alp = b["rollout_log_probs"], b["old_log_probs"]
    if "response_mask" in b:
        mask = b["response_mask"]
    elif "attention_mask" in b:
        mask = b["attention_mask"]
    else:
        mask = torch.ones_like(rlp)
    R = b["responses"].size(1)
    m = mask[:, -R:].bool()
    pa, pr = torch.exp(alp), torch.exp(rlp)
    if pa.shape == pr.shape == m.shape:
        a, r = torch.masked_select(pa, m), torch.masked_select(pr, m)
        corr = torch.corrcoef(torch.stack([a, r], dim=0))[0][1]
    else:  # metrics.py:47-49
        corr = torch.zeros(())
    diff = torch.masked_select(torch.abs(pa - pr), m)
    vals = torch.stack([diff.max(), diff.mean(), diff.std(), corr.to(diff.device, diff.dtype)]).tolist()
    return {"training/rollout_probs_diff_valid": 1, "training/rollout_probs_diff_max": vals[0],
            "training/rollout_probs_diff_mean": vals[1], "training/rollout_probs_diff_std": vals[2],
            "training/rollout_actor_probs_pearson_corr": vals[3]}
