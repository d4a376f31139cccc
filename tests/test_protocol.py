"""DataProto semantics on CPU (modeled on the reference's tests/test_protocol_on_cpu.py)."""

import numpy as np
import pytest
import torch

from dots.rl_amd.protocol import DataProto, TensorBatch, _union_batch, _union_numpy


def test_union_tensor_batch():
    obs = torch.randn(100, 10)
    d1 = TensorBatch({"obs": obs, "act": torch.randn(100, 3)})
    d2 = TensorBatch({"obs": obs, "next_obs": torch.randn(100, 10), "rew": torch.randn(100)})
    d3 = TensorBatch({"obs": obs.clone(), "next_obs": torch.randn(100, 10), "rew": torch.randn(100)})
    _union_batch(d1, d2)
    assert set(d1) == {"obs", "act", "next_obs", "rew"}
    with pytest.raises(AssertionError):
        _union_batch(d1, d3)


def test_union_numpy_nan_and_objects():
    data = np.random.random(100)
    nan_obj = np.array([float("nan")] * 99 + ["nan"], dtype=object)
    d1 = {"a": data, "b": nan_obj}
    _union_numpy(d1, {"a": data.copy(), "b": nan_obj.copy()})
    with pytest.raises(AssertionError):
        _union_numpy(d1, {"a": np.random.random(100)})
    arr = np.arange(24, dtype=np.int32).reshape(2, 3, 4)
    _union_numpy({"x": arr}, {"x": arr.copy()})
    with pytest.raises(AssertionError, match="not the same object"):
        _union_numpy({"x": arr}, {"x": arr + 1})


def make(n=8):
    return DataProto.from_dict({"obs": torch.arange(n * 2).view(n, 2), "rew": torch.arange(n).float()},
                               {"uid": np.array([f"u{i // 2}" for i in range(n)], dtype=object)}, {"k": 1})


def test_chunk_concat_roundtrip():
    d = make(8)
    parts = d.chunk(4)
    assert [len(p) for p in parts] == [2, 2, 2, 2]
    assert parts[1].batch["obs"].tolist() == [[4, 5], [6, 7]]
    assert list(parts[3].non_tensor_batch["uid"]) == ["u3", "u3"]
    back = DataProto.concat(parts)
    assert torch.equal(back.batch["obs"], d.batch["obs"])
    assert list(back.non_tensor_batch["uid"]) == list(d.non_tensor_batch["uid"])
    assert back.meta_info == {"k": 1}
    with pytest.raises(AssertionError):
        make(6).chunk(4)


def test_pop_select_rename():
    d = make(4)
    popped = d.pop(batch_keys=["rew"], non_tensor_batch_keys=["uid"], meta_info_keys=["k"])
    assert set(popped.batch) == {"rew"} and "uid" in popped.non_tensor_batch and popped.meta_info == {"k": 1}
    assert set(d.batch) == {"obs"} and d.non_tensor_batch == {} and d.meta_info == {}
    e = make(4).select(batch_keys=["obs"], non_tensor_batch_keys=[])
    assert set(e.batch) == {"obs"} and e.non_tensor_batch == {}
    f = make(4).rename("rew", "reward")
    assert "reward" in f.batch and "rew" not in f.batch


def test_repeat_interleave_and_tile():
    d = DataProto.from_dict({"x": torch.tensor([[1, 2], [3, 4]])}, {"l": np.array(["a", "b"], dtype=object)})
    r = d.repeat(2, interleave=True)
    assert r.batch["x"].tolist() == [[1, 2], [1, 2], [3, 4], [3, 4]]
    assert list(r.non_tensor_batch["l"]) == ["a", "a", "b", "b"]
    t = d.repeat(2, interleave=False)
    assert t.batch["x"].tolist() == [[1, 2], [3, 4], [1, 2], [3, 4]]
    assert list(t.non_tensor_batch["l"]) == ["a", "b", "a", "b"]


def test_reorder_and_index():
    d = make(4)
    d.reorder(torch.tensor([3, 2, 1, 0]))
    assert d.batch["rew"].tolist() == [3.0, 2.0, 1.0, 0.0]
    assert list(d.non_tensor_batch["uid"]) == ["u1", "u1", "u0", "u0"]
    e = make(6)
    assert len(e[1:4]) == 3 and e[1:4].batch["rew"].tolist() == [1.0, 2.0, 3.0]
    assert e[[0, 5]].batch["rew"].tolist() == [0.0, 5.0]
    assert e[np.array([1, 2])].batch["rew"].tolist() == [1.0, 2.0]
    m = torch.tensor([True, False, True, False, False, True])
    assert e[m].batch["rew"].tolist() == [0.0, 2.0, 5.0]
    assert len(e[2]) == 1
    assert [len(s) for s in e.split(4)] == [4, 2]


def test_union_dataproto_and_no_batch_len():
    d = make(4)
    other = DataProto.from_dict({"obs": d.batch["obs"], "adv": torch.zeros(4)}, meta_info={"t": 2})
    d.union(other)
    assert set(d.batch) == {"obs", "rew", "adv"} and d.meta_info == {"k": 1, "t": 2}
    nb = DataProto.from_dict(non_tensors={"uid": np.array(["a", "b", "c"], dtype=object)})
    assert len(nb) == 3
    # the driver pops all prompt tensors, repeats the uid-only batch and unions rollout output into it
    ids = DataProto.from_dict({"input_ids": torch.zeros(2, 3)}, {"uid": np.array(["p", "q"], dtype=object)})
    ids.pop(batch_keys=["input_ids"])
    rep = ids.repeat(2, interleave=True)
    assert len(rep) == 4
    rep.union(DataProto.from_dict({"responses": torch.ones(4, 5)}))
    assert rep.batch["responses"].shape == (4, 5)


def test_batch_size_consistency_is_enforced():
    with pytest.raises(ValueError):
        TensorBatch({"a": torch.zeros(3), "b": torch.zeros(4)})
    with pytest.raises(AssertionError):
        DataProto.from_dict({"a": torch.zeros(3)}, {"u": np.array([1, 2], dtype=object)})
