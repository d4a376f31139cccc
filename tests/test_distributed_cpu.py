"""The N>1 data-parallel path on CPU: world_size-2 gloo groups (127.0.0.1 rendezvous).

* SPMD WorkerGroup dispatch/collect: each rank computes its DP chunk, the all-gather returns the full
  batch in rank order on every rank (decorator.py:213-312 chunk / concat semantics);
* ONE_TO_ALL / RANK_ZERO dispatch;
* DataProto.all_gather of tensors + non-tensor (uid) arrays;
* gradient averaging of the flat buffer (the RCCL all-reduce of FlatAdamW.step, AVG) on gloo, and its
  overlapped per-layer form (async all-reduce per decoder layer from the backward hook).
"""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(rank, world, port, fn, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, fn(rank, world)))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def spawn(fn, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_run, args=(r, world, port, fn, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    return out


def _worker_group_case(rank, world):
    from dots.rl_amd.protocol import DataProto
    from dots.rl_amd.single_controller import (Dispatch, SPMDWorkerGroup, Worker,
                                               make_nd_compute_dataproto_dispatch_fn, register)

    class W(Worker):
        @register(dispatch_mode=make_nd_compute_dataproto_dispatch_fn(mesh_name="actor"))
        def double(self, data: DataProto):
            return DataProto.from_dict({"y": data.batch["x"] * 2, "who": torch.full((len(data),), self.rank)})

        @register(dispatch_mode=Dispatch.ONE_TO_ALL)
        def hello(self, v):
            return (self.rank, v)

        @register(dispatch_mode=Dispatch.RANK_ZERO)
        def only0(self):
            return "zero"

    wg = SPMDWorkerGroup(W())
    data = DataProto.from_dict({"x": torch.arange(8).float()}, {"uid": np.array([f"u{i}" for i in range(8)], dtype=object)})
    out = wg.double(data)
    gathered = data.all_gather()  # replicated input -> world copies
    return {"y": out.batch["y"].tolist(), "who": out.batch["who"].tolist(), "hello": wg.hello(5),
            "only0": wg.only0(), "gathered_len": len(gathered), "gathered_uid": list(gathered.non_tensor_batch["uid"])}


def test_spmd_worker_group_dispatch_collect():
    out = spawn(_worker_group_case)
    for r in (0, 1):
        o = out[r]
        assert not isinstance(o, str), o
        assert o["y"] == [2.0 * i for i in range(8)]
        assert o["who"] == [0] * 4 + [1] * 4  # rank r computed chunk r; the collect is in rank order
        assert o["hello"] == [(r, 5)]
        assert o["gathered_len"] == 16 and o["gathered_uid"][:8] == [f"u{i}" for i in range(8)]
    assert out[0]["only0"] == "zero" and out[1]["only0"] is None


def _grad_avg_case(rank, world):
    g = torch.full((1000,), float(rank + 1))
    dist.all_reduce(g, op=dist.ReduceOp.AVG)
    return g[:3].tolist()


def test_flat_gradient_average():
    out = spawn(_grad_avg_case)
    assert out[0] == out[1] == [1.5, 1.5, 1.5]


def _overlap_case(rank, world):
    import types

    from dots.rl_amd.dp_actor import FlatAdamW
    from dots.rl_amd.qwen2 import ParamStore, Qwen2Config

    cfg = Qwen2Config.from_dict(dict(vocab_size=64, hidden_size=32, intermediate_size=64, num_hidden_layers=3,
                                     num_attention_heads=2, num_key_value_heads=1, max_position_embeddings=64,
                                     tie_word_embeddings=True))
    store = ParamStore(cfg, "cpu", compute_dtype=torch.float32, trainable=True)
    g = torch.Generator().manual_seed(rank)
    store.grad.copy_(torch.randn(store.grad.shape, generator=g))
    want = store.grad.clone()
    dist.all_reduce(want, op=dist.ReduceOp.AVG)  # the monolithic form
    opt = FlatAdamW(store, lr=1e-3)
    model = types.SimpleNamespace(grad_ready_hook=None)
    opt.begin_overlap(model)
    for i in reversed(range(cfg.num_hidden_layers)):  # backward order: last layer first
        model.grad_ready_hook(i)
    opt.end_overlap(model)
    assert model.grad_ready_hook is None
    opt.allreduce_grads()
    ranges = [store.layer_range(i) for i in range(cfg.num_hidden_layers)]
    return dict(equal=bool(torch.equal(store.grad, want)), ranges=ranges, n=store.grad.numel())


def test_overlapped_gradient_allreduce_matches_monolithic():
    """FlatAdamW's per-layer async all-reduce (started from the layer backward hook of the last micro-batch)
    plus the rest-of-buffer all-reduce averages exactly what one all-reduce of the flat gradient does."""
    out = spawn(_overlap_case)
    assert out[0]["equal"] and out[1]["equal"]
    ranges = out[0]["ranges"]
    assert all(a < b for a, b in ranges) and all(ranges[k][1] <= ranges[k + 1][0] for k in range(len(ranges) - 1))
    # norm weights (small region) and the embedding before the first layer; nothing of a layer past the end
    assert ranges[0][0] > 0 and ranges[-1][1] <= out[0]["n"]


def test_config_overrides():
    from dots.rl_amd.config import apply_overrides, default_config

    cfg = default_config()
    apply_overrides(cfg, ["actor_rollout_ref.actor.ppo_mini_batch_size=16", "algorithm.adv_estimator=gae",
                          "actor_rollout_ref.rollout.top_p=0.9", "trainer.logger=['console']",
                          "+actor_rollout_ref.model.override_config.num_hidden_layers=2",
                          "actor_rollout_ref.actor.clip_ratio_high=null"])
    assert cfg.actor_rollout_ref.actor.ppo_mini_batch_size == 16
    assert cfg.algorithm.adv_estimator == "gae"
    assert cfg.actor_rollout_ref.rollout.top_p == 0.9
    assert cfg.trainer.logger == ["console"]
    assert cfg.actor_rollout_ref.model.override_config.num_hidden_layers == 2
    assert cfg.actor_rollout_ref.actor.clip_ratio_high is None
    with pytest.raises(KeyError):
        apply_overrides(cfg, ["actor_rollout_ref.actor.no_such_key=1"])
