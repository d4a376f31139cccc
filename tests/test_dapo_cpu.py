"""DAPO recipe host logic on CPU (config #5): the overlong-buffer reward vs the reference DAPORewardManager's
vectors (tests/golden/dapo_reward.npz), the dynamic-sampling group filter (dapo_ray_trainer.py:213-244), and
the recipe's generation loop (accumulate filtered groups until train_batch_size prompts, cut to B*n)."""

import numpy as np
import pytest
import torch

from dots.rl_amd.config import AttrDict, apply_overrides, default_config, to_attr
from dots.rl_amd.dapo_trainer import RayDAPOTrainer, dapo_overrides, filter_groups
from dots.rl_amd.protocol import DataProto
from dots.rl_amd.reward import DAPOSyntheticRewardManager


def test_overlong_reward_matches_reference(golden):
    z, meta = golden("dapo_reward.npz")
    for ci, c in enumerate(meta["cases"]):
        ob = to_attr(dict(enable=True, len=c["overlong_len"], penalty_factor=c["penalty_factor"], log=True))
        rm = DAPOSyntheticRewardManager(max_resp_len=c["max_resp_len"], overlong_buffer_cfg=ob)
        acc = torch.from_numpy(z[f"c{ci}_acc"])
        rm._scores = lambda data, acc=acc: acc  # the reference's compute_score results for these rows
        data = DataProto.from_dict({"responses": torch.from_numpy(z[f"c{ci}_responses"]),
                                    "attention_mask": torch.from_numpy(z[f"c{ci}_attention_mask"])})
        out = rm(data, return_dict=True)
        np.testing.assert_array_equal(out["reward_tensor"].numpy(), z[f"c{ci}_reward_tensor"])
        np.testing.assert_array_equal(out["reward_extra_info"]["overlong_reward"], z[f"c{ci}_overlong_reward"])
        np.testing.assert_array_equal(out["reward_extra_info"]["acc"], z[f"c{ci}_acc"])


def _batch(uids, vals):
    B = len(uids)
    d = DataProto.from_dict({"token_level_rewards": torch.tensor(vals, dtype=torch.float32)[:, None].repeat(1, 3),
                             "responses": torch.arange(B)[:, None].repeat(1, 3)},
                            non_tensors={"uid": np.array(uids, dtype=object), "acc": np.array(vals)})
    return d


def test_filter_groups_keeps_groups_with_spread():
    uids = ["a", "a", "b", "b", "c", "d", "d", "d"]
    vals = [1.0, 0.0, 1.0, 1.0, 0.0, 0.0, 0.0, 0.5]
    kept, n = filter_groups(_batch(uids, vals), "acc")
    assert kept == [0, 1, 4, 5, 6, 7] and n == 3  # "b" has zero spread; the singleton "c" stays
    kept2, n2 = filter_groups(_batch(uids, vals), "seq_final_reward")  # row sums = 3 * val: same decision
    assert kept2 == kept and n2 == n


class _FakeTrainer(RayDAPOTrainer):
    """Drives RayDAPOTrainer.step's generation loop without workers: each 'rollout' returns a scored batch of
    pre-set per-prompt outcomes; _train_on records what it received."""

    def __init__(self, cfg, outcomes):
        self.config = cfg
        self.reward_fn = lambda data, return_dict=True: {"reward_tensor": data.batch["preset"].clone(),
                                                         "reward_extra_info": {"acc": data.batch["preset"].sum(-1).numpy()}}
        self.outcomes = list(outcomes)
        self.global_steps = 1
        self.n_gpus = 1
        self.use_critic = False
        self.trained = None
        self.train_dataloader = AttrDict(next=lambda: {})

    def _rollout(self, src, timing_raw):
        acc = self.outcomes.pop(0)  # (prompts, n) 0/1 outcomes
        P, n = acc.shape
        uids = self._uids(P)
        preset = torch.zeros(P * n, 4)
        preset[:, -1] = torch.tensor(acc.reshape(-1), dtype=torch.float32)
        return DataProto.from_dict({"preset": preset, "responses": torch.zeros(P * n, 4, dtype=torch.int64)},
                                   non_tensors={"uid": np.repeat(uids, n)})

    def _train_on(self, batch, metrics, timing_raw):
        self.trained = batch
        metrics["actor/entropy"] = 0.0
        return batch

    def _finish_metrics(self, batch, metrics, timing_raw):
        return metrics


def test_dynamic_sampling_accumulates_until_full():
    cfg = apply_overrides(default_config(), dapo_overrides(256) + ["data.train_batch_size=3",
                                                                     "actor_rollout_ref.rollout.n=2"])
    outcomes = [np.array([[1, 1], [0, 1], [0, 0]]),  # 1 prompt with spread
                np.array([[1, 0], [1, 1], [0, 1]])]  # 2 more -> 3 = train_batch_size
    tr = _FakeTrainer(cfg, outcomes)
    m = tr.step(batch_dict={})
    assert m["train/num_gen_batches"] == 2
    b = tr.trained
    assert len(b) == 6  # train_batch_size * n
    acc = b.batch["token_level_rewards"][:, -1].view(3, 2)
    assert ((acc[:, 0] != acc[:, 1])).all()  # only groups with spread survive
    assert len(set(b.non_tensor_batch["uid"])) == 3


def test_dynamic_sampling_gives_up_after_max_gen_batches():
    cfg = apply_overrides(default_config(), dapo_overrides(256) + ["data.train_batch_size=4",
                                                                     "actor_rollout_ref.rollout.n=2",
                                                                     "algorithm.filter_groups.max_num_gen_batches=2"])
    tr = _FakeTrainer(cfg, [np.ones((4, 2)), np.ones((4, 2))])
    with pytest.raises(ValueError, match="Generated too many"):
        tr.step(batch_dict={})
