"""DataProto — the batch container of the actor-learner boundary (mirror of verl/protocol.py:270-1072).

Same contract as the reference: ``batch`` (a dict of tensors sharing dim 0), ``non_tensor_batch`` (dict of
numpy object arrays with the same dim 0, e.g. ``uid``) and ``meta_info`` (plain dict), with the
chunk / split / concat / repeat / union / select / pop / reorder / to semantics the driver and workers rely on.

MI355X-first difference: tensordict is not used. ``TensorBatch`` is a thin dict of device tensors, so a
batch stays resident in HBM between pipeline stages instead of being pickled through an object store
(``protocol.py:330-354`` in the reference); ``all_gather`` collects rank shards with RCCL/gloo collectives.
"""

from __future__ import annotations

import copy
from dataclasses import dataclass, field
from typing import Any

import numpy as np
import torch


class TensorBatch(dict):
    """dict[str, Tensor] whose values share ``batch_size`` along dim 0 (the TensorDict subset in use)."""

    def __init__(self, source=None, batch_size=None):
        super().__init__(source or {})
        if batch_size is None:
            batch_size = next(iter(self.values())).shape[0] if len(self) else 0
        self.batch_size = torch.Size([int(batch_size[0] if isinstance(batch_size, (tuple, list, torch.Size)) else batch_size)])
        for k, v in self.items():
            if v.shape[0] != self.batch_size[0]:
                raise ValueError(f"key {k}: dim0 {v.shape[0]} != batch size {self.batch_size[0]}")

    def __setitem__(self, key, value):
        if isinstance(key, str):
            if len(self) and value.shape[0] != self.batch_size[0]:
                raise ValueError(f"key {key}: dim0 {value.shape[0]} != batch size {self.batch_size[0]}")
            if not len(self):
                self.batch_size = torch.Size([value.shape[0]])
            super().__setitem__(key, value)
        else:
            raise TypeError("TensorBatch keys are strings")

    def index(self, idx) -> "TensorBatch":
        out = {k: v[idx] for k, v in self.items()}
        n = next(iter(out.values())).shape[0] if out else 0
        return TensorBatch(out, batch_size=n)

    def to(self, device) -> "TensorBatch":
        return TensorBatch({k: v.to(device, non_blocking=True) for k, v in self.items()}, batch_size=self.batch_size)

    def select(self, *keys) -> "TensorBatch":
        return TensorBatch({k: self[k] for k in keys}, batch_size=self.batch_size)

    def contiguous(self):
        return TensorBatch({k: v.contiguous() for k, v in self.items()}, batch_size=self.batch_size)


def _union_batch(a: TensorBatch | None, b: TensorBatch | None) -> TensorBatch | None:
    """protocol.py:105-118: same batch size; a conflicting key must hold an equal tensor."""
    if a is None:
        return b
    if b is None:
        return a
    assert a.batch_size == b.batch_size, f"batch sizes differ: {a.batch_size} vs {b.batch_size}"
    for k, v in b.items():
        if k in a:
            if a[k] is not v and not torch.equal(a[k], v):
                raise AssertionError(f"{k} in tensor_dict1 and tensor_dict2 are not the same object")
        else:
            a[k] = v
    return a


def _deep_equal(x, y) -> bool:
    """protocol.py:121-181 semantics: strict type match, NaN == NaN, object arrays compared elementwise."""
    if type(x) is not type(y):
        return False
    if isinstance(x, float):
        return (x != x and y != y) or x == y
    if isinstance(x, np.ndarray):
        if x.dtype != y.dtype or x.shape != y.shape:
            return False
        if x.dtype != object:
            return bool(np.array_equal(x, y, equal_nan=x.dtype.kind in "fc"))
        return all(_deep_equal(p, q) for p, q in zip(x.flat, y.flat))
    return bool(x == y)


def _union_numpy(a: dict, b: dict) -> dict:
    for k, v in b.items():
        if k in a:
            assert isinstance(v, np.ndarray) and isinstance(a[k], np.ndarray)
            assert a[k] is v or _deep_equal(a[k], v), f"`{k}` in tensor_dict1 and tensor_dict2 are not the same object."
        a[k] = v
    return a


def _union_meta(a: dict, b: dict) -> dict:
    for k, v in b.items():
        if k in a and a[k] is not v:
            try:
                same = a[k] == v
                same = bool(same) if not isinstance(same, (np.ndarray, torch.Tensor)) else bool(np.all(same))
            except Exception:  # noqa: BLE001
                same = False
            assert same, f"{k} in meta_info differs"
        a[k] = v
    return a


@dataclass
class DataProto:
    batch: TensorBatch | None = None
    non_tensor_batch: dict[str, np.ndarray] = field(default_factory=dict)
    meta_info: dict[str, Any] = field(default_factory=dict)

    def __post_init__(self):
        if self.batch is not None and not isinstance(self.batch, TensorBatch):
            self.batch = TensorBatch(dict(self.batch))
        self.check_consistency()

    # ------------------------------------------------------------------ construction
    @classmethod
    def from_single_dict(cls, data: dict, meta_info=None):
        tensors = {k: v for k, v in data.items() if isinstance(v, torch.Tensor)}
        non_tensors = {k: v for k, v in data.items() if isinstance(v, np.ndarray)}
        return cls.from_dict(tensors, non_tensors, meta_info)

    @classmethod
    def from_dict(cls, tensors: dict | None = None, non_tensors: dict | None = None, meta_info=None, num_batch_dims=1):
        assert num_batch_dims == 1, "only one batch dim"
        tensors = tensors or {}
        non_tensors = {k: np.asarray(v, dtype=object) if not isinstance(v, np.ndarray) else v
                       for k, v in (non_tensors or {}).items()}
        batch = TensorBatch(tensors) if tensors else None
        return cls(batch=batch, non_tensor_batch=non_tensors, meta_info=dict(meta_info or {}))

    def check_consistency(self):
        n = len(self)
        for k, v in self.non_tensor_batch.items():
            assert isinstance(v, np.ndarray), f"non_tensor_batch[{k}] must be a numpy array"
            if self.batch is not None:
                assert v.shape[0] == n, f"non_tensor_batch[{k}] has {v.shape[0]} rows, batch has {n}"

    # ------------------------------------------------------------------ size / indexing
    def __len__(self):
        if self.batch is not None and len(self.batch):
            return self.batch.batch_size[0]
        if self.non_tensor_batch:
            return next(iter(self.non_tensor_batch.values())).shape[0]
        return 0

    def __getitem__(self, item):
        if isinstance(item, slice):
            return self.slice(item.start, item.stop, item.step)
        if isinstance(item, (list, np.ndarray, torch.Tensor)):
            return self.select_idxs(item)
        if isinstance(item, (int, np.integer)):
            return DataProto(batch=self.batch.index(slice(item, item + 1)) if self.batch is not None else None,
                             non_tensor_batch={k: v[item:item + 1] for k, v in self.non_tensor_batch.items()},
                             meta_info=self.meta_info)
        raise TypeError(f"Indexing with {type(item)} is not supported")

    def slice(self, start=None, end=None, step=None):
        sl = slice(start, end, step)
        return DataProto(batch=self.batch.index(sl) if self.batch is not None else None,
                         non_tensor_batch={k: v[sl] for k, v in self.non_tensor_batch.items()},
                         meta_info=self.meta_info)

    def select_idxs(self, idxs):
        if isinstance(idxs, list):
            idxs = torch.tensor(idxs, dtype=torch.int64)
        if isinstance(idxs, np.ndarray):
            idxs = torch.from_numpy(idxs)
        if idxs.dtype == torch.bool:
            idxs = torch.nonzero(idxs).flatten()
        idx_np = idxs.cpu().numpy()
        batch = None
        if self.batch is not None:
            batch = TensorBatch({k: v[idxs.to(v.device)] for k, v in self.batch.items()}, batch_size=len(idx_np))
        return DataProto(batch=batch, non_tensor_batch={k: v[idx_np] for k, v in self.non_tensor_batch.items()},
                         meta_info=self.meta_info)

    # ------------------------------------------------------------------ key ops
    def select(self, batch_keys=None, non_tensor_batch_keys=None, meta_info_keys=None, deepcopy=False):
        batch = self.batch.select(*batch_keys) if (batch_keys is not None and self.batch is not None) else self.batch
        ntb = ({k: v for k, v in self.non_tensor_batch.items() if k in non_tensor_batch_keys}
               if non_tensor_batch_keys is not None else self.non_tensor_batch)
        meta = {k: v for k, v in self.meta_info.items() if k in meta_info_keys} if meta_info_keys is not None else self.meta_info
        if deepcopy:
            ntb, meta = copy.deepcopy(ntb), copy.deepcopy(meta)
        return DataProto(batch=batch, non_tensor_batch=dict(ntb), meta_info=dict(meta))

    def pop(self, batch_keys=None, non_tensor_batch_keys=None, meta_info_keys=None):
        tensors = {k: self.batch.pop(k) for k in (batch_keys or [])}
        non_tensors = {k: self.non_tensor_batch.pop(k) for k in (non_tensor_batch_keys or [])}
        meta = {k: self.meta_info.pop(k) for k in (meta_info_keys or [])}
        return DataProto.from_dict(tensors, non_tensors, meta)

    def rename(self, old_keys=None, new_keys=None):
        old_keys = [old_keys] if isinstance(old_keys, str) else old_keys
        new_keys = [new_keys] if isinstance(new_keys, str) else new_keys
        assert len(old_keys) == len(new_keys)
        for o, n in zip(old_keys, new_keys):
            self.batch[n] = self.batch.pop(o)
        return self

    def union(self, other: "DataProto") -> "DataProto":
        """protocol.py:670-687 — in-place union of batch, non-tensor batch and meta_info."""
        self.batch = _union_batch(self.batch, other.batch)
        self.non_tensor_batch = _union_numpy(self.non_tensor_batch, other.non_tensor_batch)
        self.meta_info = _union_meta(self.meta_info, other.meta_info)
        return self

    # ------------------------------------------------------------------ splitting
    def chunk(self, chunks: int) -> list["DataProto"]:
        """protocol.py:753-792 — equal chunks along dim 0 (must divide)."""
        n = len(self)
        assert n % chunks == 0, f"only support equal chunk. Got size of DataProto {n} and chunk {chunks}."
        size = n // chunks
        return [self.slice(i * size, (i + 1) * size) for i in range(chunks)]

    def split(self, split_size: int) -> list["DataProto"]:
        return [self[i:i + split_size] for i in range(0, len(self), split_size)]

    @staticmethod
    def concat(data: list["DataProto"]) -> "DataProto":
        batch = None
        if data[0].batch is not None:
            keys = list(data[0].batch.keys())
            batch = TensorBatch({k: torch.cat([d.batch[k] for d in data], dim=0) for k in keys})
        ntb = {k: np.concatenate([d.non_tensor_batch[k] for d in data], axis=0) for k in data[0].non_tensor_batch}
        return DataProto(batch=batch, non_tensor_batch=ntb, meta_info=data[0].meta_info)

    def reorder(self, indices):
        """In place (protocol.py:828-834)."""
        idx_np = indices.detach().cpu().numpy()
        self.batch = TensorBatch({k: v[indices.to(v.device)] for k, v in self.batch.items()}, batch_size=len(idx_np))
        self.non_tensor_batch = {k: v[idx_np] for k, v in self.non_tensor_batch.items()}

    def repeat(self, repeat_times=2, interleave=True):
        """protocol.py:836-878."""
        batch = None
        if self.batch is not None:
            if interleave:
                rep = {k: v.repeat_interleave(repeat_times, dim=0) for k, v in self.batch.items()}
            else:
                rep = {k: v.unsqueeze(0).expand(repeat_times, *v.shape).reshape(-1, *v.shape[1:]) for k, v in self.batch.items()}
            batch = TensorBatch(rep, batch_size=len(self) * repeat_times)
        ntb = {}
        for k, v in self.non_tensor_batch.items():
            ntb[k] = np.repeat(v, repeat_times, axis=0) if interleave else np.tile(v, (repeat_times,) + (1,) * (v.ndim - 1))
        return DataProto(batch=batch, non_tensor_batch=ntb, meta_info=self.meta_info)

    def to(self, device) -> "DataProto":
        if self.batch is not None:
            self.batch = self.batch.to(device)
        return self

    # ------------------------------------------------------------------ distributed
    def all_gather(self, group=None) -> "DataProto":
        """Concatenate every rank's shard in rank order (the collect side of DP_COMPUTE_PROTO).

        Tensors go through one all_gather_into_tensor per key (RCCL on GPU tensors, gloo on CPU); the
        small non-tensor arrays through all_gather_object. Requires equal shard sizes (chunk semantics)."""
        import torch.distributed as dist

        if not dist.is_initialized() or dist.get_world_size(group) == 1:
            return self
        world = dist.get_world_size(group)
        batch = None
        if self.batch is not None:
            out = {}
            for k, v in self.batch.items():
                v = v.contiguous()
                buf = torch.empty((world * v.shape[0],) + tuple(v.shape[1:]), dtype=v.dtype, device=v.device)
                dist.all_gather_into_tensor(buf, v, group=group)
                out[k] = buf
            batch = TensorBatch(out, batch_size=world * len(self))
        ntb = {}
        if self.non_tensor_batch:
            objs = [None] * world
            dist.all_gather_object(objs, self.non_tensor_batch, group=group)
            ntb = {k: np.concatenate([o[k] for o in objs], axis=0) for k in self.non_tensor_batch}
        return DataProto(batch=batch, non_tensor_batch=ntb, meta_info=self.meta_info)
