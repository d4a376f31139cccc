"""Fused micro-batch execution planning (dp_actor.exec_groups / balanced_groups): grouping never reorders or
drops micro-batches, groups are near-equal, and the activation budget sets the group size. CPU only."""
import torch

from dots.rl_amd.config import QWEN25_05B
from dots.rl_amd.dp_actor import balanced_groups, exec_groups
from dots.rl_amd.protocol import DataProto
from dots.rl_amd.qwen2 import Qwen2Config


def test_balanced_groups_sizes():
    items = list(range(32))
    for n, want in ((17, [16, 16]), (16, [16, 16]), (5, [5, 5, 5, 5, 4, 4, 4]), (1, [1] * 32), (64, [32])):
        g = balanced_groups(items, n)
        assert [len(x) for x in g] == want, (n, [len(x) for x in g])
        assert sum(g, []) == items  # order kept, nothing dropped
    assert balanced_groups([], 4) == []


def test_exec_groups_budget():
    cfg = Qwen2Config.from_dict(QWEN25_05B)
    mbs = [DataProto.from_dict({"input_ids": torch.zeros(8, 768, dtype=torch.int64)}) for _ in range(32)]
    assert [len(g) for g in exec_groups({"exec_micro_batches": 1}, cfg, mbs)] == [1] * 32
    assert [len(g) for g in exec_groups({"exec_micro_batches": 8}, cfg, mbs)] == [8] * 4
    # 24 layers x 46336 B per token x 6144 tokens = 6.8 GB per micro-batch: 110 GB -> 16 per pass
    assert [len(g) for g in exec_groups({"exec_micro_batches": 0, "exec_activation_gb": 110}, cfg, mbs)] == [16, 16]
    assert [len(g) for g in exec_groups({"exec_micro_batches": 0, "exec_activation_gb": 40}, cfg, mbs)] == [6, 6, 5, 5, 5, 5]
    # prefix sharing: 7 of every 8 rows' first 511 of 768 tokens are copies (58 % of the tokens) -> 529 KB per
    # padded token: the 32 micro-batches fit one pass
    shared = 224 * 511 / (256 * 768)
    assert [len(g) for g in exec_groups({"exec_micro_batches": 0, "exec_activation_gb": 110}, cfg, mbs,
                                        shared)] == [32]
