"""The verl-side plug point as code: this package's workers behind verl's own Worker / @register / DataProto.

A verl (dots.rl) checkout selects the hot path with one branch in ``main_ppo.py:114-135`` (actor) and
``:153-172`` (critic)::

    elif config.actor_rollout_ref.actor.strategy == "mi355x":
        from dots.rl_amd.verl_adapter import MI355XActorRolloutRefWorker as ActorRolloutRefWorker
        ray_worker_group_cls = RayWorkerGroup

and one branch in ``monkey_patch.py:148-192`` for ``model.fused_kernel_options.impl_backend == "hip"``
(``patch_forward_with_backends`` below, ``forward_with_hip_backend`` as the patched forward).

The adapter classes subclass verl's ``Worker`` and re-export every hot-path method under verl's
``@register`` with the dispatch mode the reference FSDP worker uses for it (``fsdp_workers.py:571-921``,
``:1003-1340``), so Ray's dispatch / collect and the trainer are unchanged. Each call converts the verl
DataProto (TensorDict batch) into this package's DataProto with the same keys, dtypes and meta_info, runs the
MI355X worker, and converts back with the tensors on the CPU as the reference returns them
(``fsdp_workers.py:716,759,794,832``).

verl, ray and tensordict are imported lazily: this module imports without them, and the classes are
built on first attribute access (``MI355XActorRolloutRefWorker``, ``MI355XCriticWorker``).
"""

from __future__ import annotations

import functools

import torch

from . import protocol

ACTOR_METHODS = {  # name -> (dispatch, mesh) as fsdp_workers.ActorRolloutRefWorker registers them
    "init_model": ("one_to_all", None),
    "generate_sequences": ("nd", "rollout"),
    "compute_log_prob": ("nd", "actor"),
    "compute_ref_log_prob": ("nd", "actor"),
    "update_actor": ("nd", "actor"),
    "save_checkpoint": ("one_to_all", None),
    "load_checkpoint": ("one_to_all", None),
    "start_profile": ("one_to_all", None),  # fsdp_workers.py:913-921 (DistProfilerExtension)
    "stop_profile": ("one_to_all", None),
}
CRITIC_METHODS = {  # fsdp_workers.CriticWorker
    "init_model": ("one_to_all", None),
    "compute_values": ("nd", "critic"),
    "update_critic": ("nd", "critic"),
    "save_checkpoint": ("one_to_all", None),
    "load_checkpoint": ("one_to_all", None),
    "start_profile": ("one_to_all", None),
    "stop_profile": ("one_to_all", None),
}
_DATA_METHODS = {"generate_sequences", "compute_log_prob", "compute_ref_log_prob", "update_actor",
                 "compute_values", "update_critic"}


def to_ours(d, device=None) -> protocol.DataProto:
    """verl DataProto -> dots.rl_amd DataProto: same tensor keys / dtypes, non-tensor arrays and meta_info."""
    tensors = {k: (v.to(device) if device is not None else v) for k, v in d.batch.items()} if d.batch is not None else {}
    return protocol.DataProto.from_dict(tensors, dict(d.non_tensor_batch), dict(d.meta_info))


def to_verl(d: protocol.DataProto, device="cpu"):
    """dots.rl_amd DataProto -> verl DataProto (tensors moved to ``device``, the reference's CPU return)."""
    from verl import DataProto as VerlDataProto

    if d.batch is None:
        return VerlDataProto(batch=None, non_tensor_batch=dict(d.non_tensor_batch), meta_info=dict(d.meta_info))
    tensors = {k: v.to(device) for k, v in d.batch.items()}
    return VerlDataProto.from_dict(tensors=tensors, non_tensors=dict(d.non_tensor_batch), meta_info=dict(d.meta_info))


def _dispatch_mode(kind, mesh):
    from verl.single_controller.base.decorator import Dispatch, make_nd_compute_dataproto_dispatch_fn

    return Dispatch.ONE_TO_ALL if kind == "one_to_all" else make_nd_compute_dataproto_dispatch_fn(mesh_name=mesh)


def _make_cls(name, impl_factory, methods, meshes):
    from verl.single_controller.base import Worker
    from verl.single_controller.base.decorator import register

    def __init__(self, config, *args, **kwargs):
        Worker.__init__(self)
        self.impl = impl_factory(config, *args, **kwargs)
        import torch.distributed as dist

        rank = dist.get_rank() if dist.is_initialized() else 0
        for mesh in meshes:
            self._register_dispatch_collect_info(mesh, dp_rank=rank, is_collect=True)

    ns = {"__init__": __init__, "__doc__": f"verl Worker around dots.rl_amd ({name}); see verl_adapter."}
    for meth, (kind, mesh) in methods.items():
        def make(meth=meth):
            if meth in _DATA_METHODS:
                def call(self, data):
                    return to_verl(getattr(self.impl, meth)(to_ours(data, self.impl.device)))
            else:
                def call(self, *a, **k):
                    return getattr(self.impl, meth)(*a, **k)
            call.__name__ = meth
            return register(dispatch_mode=_dispatch_mode(kind, mesh))(call)

        ns[meth] = make()
    return type(name, (Worker,), ns)


@functools.lru_cache(maxsize=None)
def make_actor_rollout_ref_worker_cls():
    from .workers import ActorRolloutRefWorker

    return _make_cls("MI355XActorRolloutRefWorker",
                     lambda config, role="actor_rollout_ref", **kw: ActorRolloutRefWorker(config, role=role, **kw),
                     ACTOR_METHODS, ("actor", "rollout"))


@functools.lru_cache(maxsize=None)
def make_critic_worker_cls():
    from .workers import CriticWorker

    return _make_cls("MI355XCriticWorker", lambda config, **kw: CriticWorker(config, **kw), CRITIC_METHODS,
                     ("critic",))


def __getattr__(name):  # PEP 562: the classes exist once verl is importable
    if name == "MI355XActorRolloutRefWorker":
        return make_actor_rollout_ref_worker_cls()
    if name == "MI355XCriticWorker":
        return make_critic_worker_cls()
    raise AttributeError(name)


# ----------------------------------------------------------------------------------- fused-kernel backend "hip"
def forward_with_hip_backend(self, input_ids=None, attention_mask=None, position_ids=None, past_key_values=None,
                             inputs_embeds=None, labels=None, use_cache=None, output_attentions=None,
                             output_hidden_states=None, return_dict=None, cache_position=None, logits_to_keep=0,
                             temperature: float = 1.0, **loss_kwargs):
    """dense_common.py:71-130 (forward_with_torch_backend) with the A21 HIP kernel (csrc/fused_linear.hip) in
    place of FusedLinearForPPO: the HF base model's last hidden states, labels rolled by one, log-probs and
    entropy over the vocabulary without writing the (B, T, V) logits."""
    from .torch_functional import fused_linear_logprob_entropy

    outputs = self.model(input_ids=input_ids, attention_mask=attention_mask, position_ids=position_ids,
                         past_key_values=past_key_values, inputs_embeds=inputs_embeds, use_cache=use_cache,
                         output_attentions=output_attentions, output_hidden_states=output_hidden_states,
                         cache_position=cache_position)
    hidden_states = outputs[0]
    if not return_dict:
        raise NotImplementedError("forward_with_hip_backend has to return_dict")
    if labels is not None:
        rolled = torch.roll(labels, shifts=-1, dims=-1)
    elif input_ids is not None:
        rolled = torch.roll(input_ids, shifts=-1, dims=-1)
    else:
        raise RuntimeError("To use forward_with_hip_backend, either labels or input_ids must be provided.")
    B, T, H = hidden_states.shape
    logp, ent = fused_linear_logprob_entropy(hidden_states.reshape(B * T, H), self.lm_head.weight,
                                             rolled.reshape(-1), temperature=temperature, calculate_entropy=True)
    from verl.models.transformers.dense_common import CausalLMOutputForPPO

    return CausalLMOutputForPPO(log_probs=logp.view(B, T), entropy=ent.view(B, T),
                                past_key_values=outputs.past_key_values, hidden_states=outputs.hidden_states,
                                attentions=outputs.attentions)


def patch_forward_with_backends(model, use_fused_kernels: bool = False, fused_kernels_backend: str | None = None):
    """monkey_patch.py:148-192 plus the "hip" backend; other backends go to the reference's own function."""
    if use_fused_kernels and fused_kernels_backend == "hip":
        model.__class__.forward = forward_with_hip_backend
        print(f"Using HIP (MI355X) backend for fused kernels in {model.__class__.__name__}")
        return
    from verl.models.transformers.monkey_patch import patch_forward_with_backends as ref_patch

    ref_patch(model, use_fused_kernels=use_fused_kernels, fused_kernels_backend=fused_kernels_backend)


__all__ = ["to_ours", "to_verl", "make_actor_rollout_ref_worker_cls", "make_critic_worker_cls",
           "forward_with_hip_backend", "patch_forward_with_backends", "ACTOR_METHODS", "CRITIC_METHODS"]
