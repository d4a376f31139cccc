"""Sequence-length balancing and dynamic micro-batching (mirror of verl/utils/seqlen_balancing.py:26-375).

Host-side planning over B integers (the attention-mask row sums): which rows form which micro-batch
(``use_dynamic_bsz``: micro-batches bounded by a token budget instead of a row count) and which rows go to
which DP rank (``trainer.balance_batch``). The partitions are the reference's exactly — same largest-
differencing (Karmarkar-Karp) merge order and tie-breaks — so micro-batch composition, and with it every
per-micro-batch token-mean, matches. Tensor work stays on the device: rows are gathered with one
index_select per key.
"""

from __future__ import annotations

import heapq
from itertools import chain

import torch
import torch.distributed as dist

from .protocol import DataProto, TensorBatch


class _Bucket:
    """One partition under construction: (sum, items) ordered as seqlen_balancing.py:28-46 orders its sets."""

    __slots__ = ("total", "items")

    def __init__(self):
        self.total = 0
        self.items = []  # (index, seqlen) in insertion order

    def key(self):
        return (self.total, len(self.items), self.items)


class _Partial:
    """k buckets kept in decreasing bucket order; heap order = largest spread first (seqlen_balancing.py:48-93)."""

    __slots__ = ("buckets",)

    def __init__(self, items, k):
        self.buckets = [_Bucket() for _ in range(k)]
        for b, (idx, n) in zip(self.buckets, items):
            b.items.append((idx, n))
            b.total += n
        self._sort()

    def _sort(self):
        self.buckets.sort(key=_Bucket.key, reverse=True)

    def spread(self):
        return self.buckets[0].total - self.buckets[-1].total

    def absorb(self, other):
        """Pair the largest bucket of self with the smallest of other, and so on, then re-sort."""
        k = len(self.buckets)
        for i in range(k):
            src = other.buckets[k - 1 - i]
            self.buckets[i].items.extend(src.items)
            self.buckets[i].total += src.total
        self._sort()

    def __lt__(self, other):
        if self.spread() != other.spread():
            return self.spread() > other.spread()
        return self.buckets[0].key() > other.buckets[0].key()


def karmarkar_karp(seqlen_list: list[int], k_partitions: int, equal_size: bool) -> list[list[int]]:
    """Largest differencing method (seqlen_balancing.py:26-127): partitions of indices, unsorted."""
    ordered = sorted((n, i) for i, n in enumerate(seqlen_list))
    heap = []
    if equal_size:
        assert len(seqlen_list) % k_partitions == 0, f"{len(seqlen_list)} % {k_partitions} != 0"
        for off in range(0, len(ordered), k_partitions):
            heapq.heappush(heap, _Partial([(i, n) for n, i in ordered[off:off + k_partitions]], k_partitions))
    else:
        for n, i in ordered:
            heapq.heappush(heap, _Partial([(i, n)], k_partitions))
    while len(heap) > 1:
        a = heapq.heappop(heap)
        b = heapq.heappop(heap)
        a.absorb(b)
        heapq.heappush(heap, a)
    parts = [[i for i, _ in b.items] for b in heap[0].buckets]
    if equal_size:
        for p in parts:
            assert len(p) * k_partitions == len(seqlen_list), f"{len(p)} * {k_partitions} != {len(seqlen_list)}"
    return parts


def get_seqlen_balanced_partitions(seqlen_list: list[int], k_partitions: int, equal_size: bool) -> list[list[int]]:
    """seqlen_balancing.py:150-191: balanced partitions, each sorted, all non-empty."""
    assert len(seqlen_list) >= k_partitions, f"number of items:[{len(seqlen_list)}] < k_partitions:[{k_partitions}]"
    parts = karmarkar_karp(seqlen_list, k_partitions, equal_size)
    assert len(parts) == k_partitions, f"{len(parts)} != {k_partitions}"
    seen = set()
    out = []
    for i, p in enumerate(parts):
        assert len(p) > 0, f"the {i}-th partition is empty"
        seen.update(p)
        out.append(sorted(p))
    assert seen == set(range(len(seqlen_list)))
    return out


def log_seqlen_unbalance(seqlen_list: list[int], partitions: list[list[int]], prefix: str) -> dict:
    """seqlen_balancing.py:194-239: min/max/diff of the per-partition token sums before (contiguous chunks)
    and after balancing."""
    k = len(partitions)
    B = len(seqlen_list)
    per = B // k
    before = [sum(seqlen_list[j * per:(j + 1) * per]) for j in range(k)]
    after = [sum(seqlen_list[i] for i in p) for p in partitions]
    return {f"{prefix}/min": min(before), f"{prefix}/max": max(before), f"{prefix}/minmax_diff": max(before) - min(before),
            f"{prefix}/balanced_min": min(after), f"{prefix}/balanced_max": max(after),
            f"{prefix}/mean": sum(before) / k}


def ceildiv(a, b):
    return -(a // -b)


def rearrange_micro_batches(batch: TensorBatch, max_token_len: int, dp_group=None, num_batches_divided_by=None,
                            same_micro_num_in_dp=True, min_num_micro_batch=None, use_dynamic_bsz_balance=True):
    """seqlen_balancing.py:250-319: micro-batches whose attention-mask token sums stay near max_token_len (the
    count is the ceil of total / budget, synchronised to the max over DP ranks), balanced by Karmarkar-Karp,
    ordered by descending sum of squared lengths. Returns (list of TensorBatch, index lists)."""
    am = batch["attention_mask"]
    assert max_token_len >= am.shape[-1], (
        f"max_token_len must be greater than the sequence length. Got {max_token_len=} and {am.shape[-1]=}")
    lens = am.sum(dim=1)
    total = int(lens.sum().item())
    n_micro = min(len(lens), ceildiv(total, max_token_len))
    if min_num_micro_batch is not None:
        n_micro = max(min_num_micro_batch, n_micro)
    if dist.is_initialized() and same_micro_num_in_dp:
        t = torch.tensor([n_micro], device=am.device if am.is_cuda else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=dp_group)
        n_micro = int(t.item())
    if num_batches_divided_by is not None:
        n_micro = ceildiv(n_micro, num_batches_divided_by) * num_batches_divided_by
    lens = lens.tolist()
    assert n_micro <= len(lens)
    parts = get_seqlen_balanced_partitions(lens, n_micro, equal_size=False)
    if use_dynamic_bsz_balance:
        parts.sort(key=lambda p: (sum(lens[i] ** 2 for i in p), min(p) if p else 0), reverse=True)
    micro = []
    for p in parts:
        idx = torch.tensor(p, dtype=torch.int64, device=am.device)
        micro.append(TensorBatch({k: v.index_select(0, idx) for k, v in batch.items()}, batch_size=len(p)))
    return micro, parts


def get_reverse_idx(idx_map):
    rev = list(idx_map)
    for i, j in enumerate(idx_map):
        rev[j] = i
    return rev


def prepare_dynamic_batch(data: DataProto, max_token_len: int):
    """seqlen_balancing.py:340-359: (micro-batch DataProtos, index lists)."""
    batches, idx_list = rearrange_micro_batches(data.batch, max_token_len=max_token_len)
    out = []
    for b, idx in zip(batches, idx_list):
        out.append(DataProto(batch=b, non_tensor_batch={k: v[idx] for k, v in data.non_tensor_batch.items()},
                             meta_info=data.meta_info))
    return out, idx_list


def restore_dynamic_batch(data: torch.Tensor, batch_idx_list) -> torch.Tensor:
    """seqlen_balancing.py:362-375: rows back to the original order."""
    rev = torch.tensor(get_reverse_idx(list(chain.from_iterable(batch_idx_list))), dtype=torch.long, device=data.device)
    return data[rev]
