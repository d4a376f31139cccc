"""Run by tests/test_verl_adapter_cpu.py in a child process (the reference stubs it installs must not leak
into the test session): imports the reference's decorator / protocol / fsdp_workers from /root/reference
with tests/golden/_ref_stubs (SURVEY §8(c) recipe, plus inert stand-ins for peft & co.), builds the adapter
classes of dots.rl_amd.verl_adapter and checks them against the reference FSDP workers."""

import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
sys.path.insert(0, os.path.dirname(HERE))
import _ref_stubs  # noqa: E402

_ref_stubs.install()
_ref_stubs._auto_stub(["peft", "hydra", "sglang", "vllm", "flash_attn", "liger_kernel", "megatron"])

import numpy as np  # noqa: E402
import torch  # noqa: E402
from verl import DataProto as VerlDataProto  # noqa: E402
from verl.single_controller.base import Worker  # noqa: E402
from verl.single_controller.base.decorator import MAGIC_ATTR  # noqa: E402
import verl.workers.fsdp_workers as fw  # noqa: E402

from dots.rl_amd import protocol, verl_adapter  # noqa: E402


def _mode_key(m):
    if isinstance(m, dict):  # make_nd_compute_dataproto_dispatch_fn: partials over the mesh name
        return ("nd", m["dispatch_fn"].func.__name__, m["dispatch_fn"].args, m["collect_fn"].func.__name__,
                m["collect_fn"].args)
    return ("enum", m)


def check_worker(ours, ref, methods):
    assert issubclass(ours, Worker)
    for name in methods:
        a, b = getattr(getattr(ours, name), MAGIC_ATTR), getattr(getattr(ref, name), MAGIC_ATTR)
        assert _mode_key(a["dispatch_mode"]) == _mode_key(b["dispatch_mode"]), (name, a, b)
        assert a["execute_mode"] == b["execute_mode"] and a["blocking"] == b["blocking"], (name, a, b)
    print(f"{ours.__name__}: {len(methods)} methods carry the reference dispatch modes of {ref.__name__}")


def check_round_trip():
    g = torch.Generator().manual_seed(0)
    tensors = {"input_ids": torch.randint(0, 1000, (6, 9), generator=g), "attention_mask": torch.ones(6, 9, dtype=torch.int64),
               "old_log_probs": torch.randn(6, 4, generator=g), "values": torch.randn(6, 4, generator=g).bfloat16(),
               "flags": torch.rand(6, generator=g) > 0.5}
    nt = {"uid": np.array([f"u{i // 2}" for i in range(6)], dtype=object),
          "reward_model": np.array([{"ground_truth": str(i)} for i in range(6)], dtype=object)}
    meta = {"temperature": 0.7, "global_token_num": [9] * 6, "eos_token_id": 2}
    ref = VerlDataProto.from_dict(tensors=dict(tensors), non_tensors=dict(nt), meta_info=dict(meta))
    ours = verl_adapter.to_ours(ref)
    assert isinstance(ours, protocol.DataProto) and len(ours) == len(ref) == 6
    assert set(ours.batch.keys()) == set(tensors)
    for k, v in tensors.items():
        assert ours.batch[k].dtype == v.dtype and torch.equal(ours.batch[k], v), k
    assert set(ours.non_tensor_batch) == set(nt) and all((ours.non_tensor_batch[k] == nt[k]).all() for k in nt)
    assert ours.meta_info == meta
    # ours -> verl after a chunk (the dispatch path) keeps keys / dtypes / values
    back = verl_adapter.to_verl(ours.chunk(2)[1])
    assert isinstance(back, VerlDataProto) and len(back) == 3
    assert set(back.batch.keys()) == set(tensors)
    for k, v in tensors.items():
        assert back.batch[k].dtype == v.dtype and torch.equal(back.batch[k], v[3:]), k
    assert (back.non_tensor_batch["uid"] == nt["uid"][3:]).all() and back.meta_info == meta
    print("DataProto verl <-> dots.rl_amd round trip: keys, dtypes, values, non-tensors, meta_info identical")


def check_fused_backend():
    class Dummy:
        def forward(self):
            return "hf"

    m = Dummy()
    verl_adapter.patch_forward_with_backends(m, use_fused_kernels=True, fused_kernels_backend="hip")
    assert Dummy.forward is verl_adapter.forward_with_hip_backend
    import inspect

    from verl.models.transformers.dense_common import forward_with_torch_backend

    assert list(inspect.signature(verl_adapter.forward_with_hip_backend).parameters) == \
        list(inspect.signature(forward_with_torch_backend).parameters)
    print("fused_kernels_backend='hip' patches the forward; signature == dense_common.forward_with_torch_backend")


if __name__ == "__main__":
    check_worker(verl_adapter.MI355XActorRolloutRefWorker, fw.ActorRolloutRefWorker, verl_adapter.ACTOR_METHODS)
    check_worker(verl_adapter.MI355XCriticWorker, fw.CriticWorker, verl_adapter.CRITIC_METHODS)
    check_round_trip()
    check_fused_backend()
    print("OK")
