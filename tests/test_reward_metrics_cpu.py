"""A19 reward and A20 metrics against fixtures produced by the reference (tests/golden/grpo_step.npz, made by
tests/golden/make_golden.py::gen_grpo_step from a reference-composed GRPO step on the tiny Qwen2):

* NaiveRewardManager (naive.py:46-122) + gsm8k strict scoring (gsm8k.py:52) on the reference rollout's
  responses decoded by the shared stub tokenizer -> the same reward tensor, bit for bit;
* the reward-model path (rm_scores returned as the reward tensor, naive.py:55-60);
* compute_data_metrics / compute_timing_metrics / compute_throughout_metrics (metric_utils.py:80-302) on the
  reference's final batch -> the same values;
* FlopsCounter.estimate_flops (flops_counter.py:135-167) for the tiny model and Qwen2.5-0.5B -> the same TFLOP/s.
"""

import json
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
from stub_tokenizer import StubTokenizer  # noqa: E402

from dots.rl_amd.protocol import DataProto  # noqa: E402
from dots.rl_amd.reward import NaiveRewardManager, get_reward_manager_cls, load_reward_manager  # noqa: E402
from dots.rl_amd.reward_score import default_compute_score, gsm8k_compute_score, gsm8k_extract_solution  # noqa: E402


def _cases():
    z = np.load(os.path.join(HERE, "golden", "grpo_step.npz"), allow_pickle=False)
    return z, json.loads(str(z["__meta__"]))["cases"]


def _batch(z, ci, meta):
    t = lambda k: torch.from_numpy(z[f"c{ci}_{k}"])  # noqa: E731
    B = t("responses").shape[0]
    n = meta["n"]
    gts = meta["ground_truths"]
    nt = {"data_source": np.array(["openai/gsm8k"] * B, dtype=object),
          "reward_model": np.array([{"ground_truth": gts[i // n]} for i in range(B)], dtype=object),
          "uid": np.array([f"uid{g}" for g in meta["uid_groups"]], dtype=object)}
    tensors = {k: t(k) for k in ("prompts", "responses", "input_ids", "attention_mask", "position_ids",
                                 "response_mask", "old_log_probs", "ref_log_prob", "advantages", "returns",
                                 "token_level_scores")}
    tensors["token_level_rewards"] = tensors["token_level_scores"]
    d = DataProto.from_dict(tensors=tensors, non_tensors=nt)
    d.meta_info["global_token_num"] = d.batch["attention_mask"].sum(-1).tolist()
    return d


def test_gsm8k_extract_and_score():
    assert gsm8k_extract_solution("step 1 #### 12 then #### -3,000") == "-3000"
    assert gsm8k_extract_solution("no marker 42") is None
    assert gsm8k_extract_solution("no marker 42 and 7.", "flexible") == "7."
    assert gsm8k_extract_solution("x" * 400 + "#### 5") == "5"
    assert gsm8k_extract_solution("#### 5" + "x" * 400) is None  # only the final 300 characters are searched
    assert gsm8k_compute_score("#### 72", "72") == 1.0
    assert gsm8k_compute_score("#### 71", "72") == 0.0
    assert gsm8k_compute_score("72", "72") == 0
    assert default_compute_score("openai/gsm8k", "ans #### 3", "3") == 1.0
    with pytest.raises(NotImplementedError):
        default_compute_score("lighteval/MATH", "x", "y")


@pytest.mark.parametrize("ci", [0, 1])
def test_naive_reward_manager_matches_reference(ci):
    z, cases = _cases()
    meta = cases[ci]
    d = _batch(z, ci, meta)
    out = NaiveRewardManager(tokenizer=StubTokenizer(), num_examine=0)(d, return_dict=True)
    np.testing.assert_array_equal(out["reward_tensor"].numpy(), z[f"c{ci}_rule_scores"])
    # reward-model scores short-circuit the rule path (naive.py:55-60)
    d.batch["rm_scores"] = torch.from_numpy(z[f"c{ci}_token_level_scores"])
    rm = NaiveRewardManager(tokenizer=StubTokenizer(), num_examine=0)(d)
    np.testing.assert_array_equal(rm.numpy(), z[f"c{ci}_token_level_scores"])


def test_reward_registry_and_loader():
    from dots.rl_amd.config import apply_overrides, default_config

    assert get_reward_manager_cls("naive") is NaiveRewardManager
    with pytest.raises(ValueError):
        get_reward_manager_cls("nope")
    cfg = apply_overrides(default_config(), ["reward_model.reward_manager=naive"])
    assert isinstance(load_reward_manager(cfg, StubTokenizer()), NaiveRewardManager)
    with pytest.raises(ValueError):
        load_reward_manager(cfg, None)


@pytest.mark.parametrize("ci", [0, 1])
def test_step_metrics_match_reference(ci):
    from dots.rl_amd.metric_utils import compute_data_metrics, compute_throughout_metrics, compute_timing_metrics

    z, cases = _cases()
    meta = cases[ci]
    d = _batch(z, ci, meta)
    timing = {"gen": 0.5, "reward": 0.01, "old_log_prob": 0.2, "ref": 0.2, "adv": 0.01, "update_actor": 0.8,
              "step": 1.75}
    got = compute_data_metrics(d, use_critic=False)
    assert set(got) == set(meta["data_metrics"])
    for k, v in meta["data_metrics"].items():
        np.testing.assert_allclose(got[k], v, rtol=1e-6, atol=1e-7, err_msg=k)
    got = compute_timing_metrics(d, timing)
    assert set(got) == set(meta["timing_metrics"])
    for k, v in meta["timing_metrics"].items():
        np.testing.assert_allclose(got[k], v, rtol=1e-12, err_msg=k)
    got = compute_throughout_metrics(d, timing, n_gpus=1)
    assert got == pytest.approx(meta["throughput_metrics"], rel=1e-12)


def test_flops_counter_matches_reference():
    from dots.rl_amd.config import QWEN25_05B
    from dots.rl_amd.flops_counter import FlopsCounter
    from dots.rl_amd.qwen2 import Qwen2Config

    z, cases = _cases()
    meta = cases[0]
    tiny = Qwen2Config.from_dict(json.load(open(os.path.join(HERE, "golden", "tiny_qwen2", "config.json"))))
    am = z["c0_attention_mask"]
    est, _ = FlopsCounter(tiny).estimate_flops(am.sum(-1).tolist(), 0.8)
    np.testing.assert_allclose(est, meta["flops_tiny_tflops"], rtol=1e-6)
    est, _ = FlopsCounter(Qwen2Config.from_dict(QWEN25_05B)).estimate_flops([768] * 512, 1.0)
    np.testing.assert_allclose(est, meta["flops_qwen05b_768x512_tflops"], rtol=1e-12)


def test_rollout_debug_metrics_match_reference(golden):
    """rollout.calculate_log_probs' monitor: training/rollout_probs_diff_* and the Pearson correlation against the
    reference's calculate_debug_metrics (utils/debug/metrics.py:63-108) on golden debug_metrics.npz, with a
    response_mask and with only an attention_mask."""
    from dots.rl_amd.metric_utils import calculate_debug_metrics

    z, meta = golden("debug_metrics.npz")
    for ci, case in enumerate(meta["cases"]):
        keys = [k[len(f"c{ci}_"):] for k in z.files if k.startswith(f"c{ci}_")]
        got = calculate_debug_metrics(DataProto.from_dict({k: torch.from_numpy(z[f"c{ci}_{k}"]) for k in keys}))
        assert set(got) == set(case["metrics"])
        for k, v in case["metrics"].items():
            assert got[k] == pytest.approx(v, rel=1e-5, abs=1e-7), k


def test_executed_flops_counts_what_ran():
    """FlopsCounter.executed_flops (perf/mfu/actor_executed): with every row's tokens executed, no prefix sharing and
    the lm_head over every position, it equals the reference formula's dense part + this repository's attention
    pricing (4 D forward + 10 D backward per causal pair and head, against the reference's 12 D per full s^2)."""
    from dots.rl_amd.config import QWEN25_05B
    from dots.rl_amd.flops_counter import FlopsCounter
    from dots.rl_amd.qwen2 import Qwen2Config

    c = Qwen2Config.from_dict(QWEN25_05B)
    fc = FlopsCounter(c)
    B, T = 4, 768
    dense_ref = fc._estimate_qwen2_flops(B * T, [0] * B, 1.0)  # sq = 0: the dense part only (TFLOP)
    # the reference counts the embedding as a second V x H matrix; executed_flops counts only the lm_head GEMM
    emb = 6 * c.vocab_size * c.hidden_size * B * T / 1e12
    got = fc.executed_flops(tokens=B * T, attn_pairs=0, lm_rows=B * T)
    assert abs(got - (dense_ref - emb)) < 1e-9 * dense_ref
    pairs = B * T * (T + 1) // 2
    att = fc.executed_flops(attn_pairs=pairs)
    assert abs(att - 14 * c.head_dim * c.num_attention_heads * c.num_hidden_layers * pairs / 1e12) < 1e-12
