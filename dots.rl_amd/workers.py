"""ActorRolloutRefWorker for ``actor.strategy = "mi355x"`` (mirror of verl/workers/fsdp_workers.py:110-921).

Same registered methods, dispatch modes, batch-size normalisation and output keys as the FSDP worker:
``init_model``, ``generate_sequences``, ``compute_log_prob`` (-> old_log_probs, entropys),
``compute_ref_log_prob`` (-> ref_log_prob), ``update_actor`` (-> meta_info["metrics"]),
``save_checkpoint`` / ``load_checkpoint``. Parallelism is replicated-parameter data parallelism: each
rank holds the full model (0.5B fits many times over in 288 GB) and gradients are averaged with one
RCCL all-reduce per optimizer step, instead of FSDP's per-layer all-gather / reduce-scatter.
Outputs stay on the device (``output_device="cuda"``); ``output_device="cpu"`` reproduces the
reference's ``.to("cpu")`` convention for callers that need it.
"""

from __future__ import annotations

import math
import os
import time

import psutil
import torch
import torch.distributed as dist

from .config import RANDOM_MODELS
from .dp_actor import DataParallelPPOActor, FlatAdamW, lr_schedule
from .dp_critic import DataParallelPPOCritic
from .flops_counter import FlopsCounter
from .profiler import DistProfiler
from .protocol import DataProto
from .qwen2 import param_specs, ParamStore, Qwen2Config, Qwen2Model
from .rollout import MI355XRollout
from .single_controller import Dispatch, Worker, make_nd_compute_dataproto_dispatch_fn, register

def resolve_model_config(model_cfg) -> Qwen2Config:
    path = model_cfg.get("path", "random:qwen2.5-0.5b")
    over = dict(model_cfg.get("override_config", {}) or {})
    if path.startswith("random:"):  # "random:<preset>" (config.RANDOM_MODELS), default Qwen2.5-0.5B
        base = dict(RANDOM_MODELS.get(path[len("random:"):] or "qwen2.5-0.5b", RANDOM_MODELS["qwen2.5-0.5b"]))
    else:
        import json

        with open(os.path.join(path, "config.json")) as f:
            base = json.load(f)
    base.update(over)
    if path.startswith("random:"):
        # a random preset whose vocabulary the override shrank has no tokenizer behind it: its preset special ids
        # (Qwen2.5: 151643 / 151645) are past the rows, so the last row is its EOS (and, below, its pad)
        V = int(base.get("vocab_size", 0))
        for key in ("eos_token_id", "pad_token_id", "bos_token_id"):
            ids = base.get(key)
            if key not in over and ids is not None and any(
                    i >= V for i in (ids if isinstance(ids, (list, tuple)) else [ids])):
                base[key] = V - 1 if key != "pad_token_id" else None
    # tokenizer.py:21-33 (set_pad_token_id): no pad id -> the eos id (the first one of a list); Meta-Llama-3-8B's
    # config.json has none, and the Qwen default (151643) is past its 128256-row vocabulary
    eos = base.get("eos_token_id")
    eos0 = eos[0] if isinstance(eos, (list, tuple)) else eos
    if base.get("pad_token_id") is None and eos0 is not None:
        base["pad_token_id"] = eos0
    cfg = Qwen2Config.from_dict(base)
    for name, ids in (("pad_token_id", cfg.pad_token_id), ("eos_token_id", cfg.eos_token_id)):
        for i in (ids if isinstance(ids, (list, tuple)) else [ids]):
            if not (isinstance(i, int) and 0 <= i < cfg.vocab_size):
                raise ValueError(f"{name}={ids!r} is not a token of the {cfg.vocab_size}-row vocabulary ({path})")
    return cfg


class ActorRolloutRefWorker(Worker):
    def __init__(self, config, role: str = "actor_rollout_ref", output_device: str = "cuda"):
        super().__init__()
        self.config = config
        self.role = role
        self._is_actor = role in ("actor", "actor_rollout", "actor_rollout_ref")
        self._is_rollout = role in ("rollout", "actor_rollout", "actor_rollout_ref")
        self._is_ref = role in ("ref", "actor_rollout_ref")
        self.output_device = output_device
        self.device = torch.device("cuda", torch.cuda.current_device())
        dp = dist.get_world_size() if dist.is_initialized() else 1
        self.dp_size = dp
        self.dp_rank = dist.get_rank() if dist.is_initialized() else 0
        for mesh in ("actor", "rollout"):
            self._register_dispatch_collect_info(mesh, dp_rank=self.dp_rank, is_collect=True)
        # fsdp_workers.py:168-196: the actor's profiler config, else the rollout's, else the ref's
        sec = config.actor if self._is_actor else (config.rollout if self._is_rollout else config.ref)
        self.profiler = DistProfiler(rank=self.dp_rank, config=sec.get("profiler") if sec is not None else None)
        # fsdp_workers.py:209-242 batch-size normalisation (per-GPU sizes)
        a = config.actor
        if self._is_actor:
            a.ppo_mini_batch_size = a.ppo_mini_batch_size * config.rollout.n // dp
            assert a.ppo_mini_batch_size > 0
            if a.get("ppo_micro_batch_size") is not None:
                a.ppo_micro_batch_size_per_gpu = a.ppo_micro_batch_size // dp
            if a.get("ppo_micro_batch_size_per_gpu") is not None:  # None with use_dynamic_bsz
                assert a.ppo_mini_batch_size % a.ppo_micro_batch_size_per_gpu == 0, (
                    f"normalized ppo_mini_batch_size {a.ppo_mini_batch_size} should be divisible by "
                    f"ppo_micro_batch_size_per_gpu {a.ppo_micro_batch_size_per_gpu}")
        r = config.rollout
        if self._is_rollout and r.get("log_prob_micro_batch_size") is not None:
            r.log_prob_micro_batch_size_per_gpu = r.log_prob_micro_batch_size // dp
        rf = config.ref
        if self._is_ref and rf.get("log_prob_micro_batch_size") is not None:
            rf.log_prob_micro_batch_size_per_gpu = rf.log_prob_micro_batch_size // dp

    # ------------------------------------------------------------------------------------------ init
    @register(dispatch_mode=Dispatch.ONE_TO_ALL)
    def init_model(self):
        cfg = self.config
        mcfg = resolve_model_config(cfg.model)
        self.model_config = mcfg
        self.flops_counter = FlopsCounter(mcfg)
        dtype = torch.float32 if cfg.model.get("dtype", "bfloat16") == "float32" else torch.bfloat16
        seed = int(cfg.model.get("seed", 1234))
        shard = _shard_spec(cfg.actor, mcfg, self.dp_rank, self.dp_size) if self._is_actor else None
        self.store = ParamStore(mcfg, self.device, compute_dtype=dtype, trainable=self._is_actor, shard=shard)
        path = cfg.model.get("path", "random:")
        if path.startswith("random:"):
            self.store.init_random(seed)
        else:
            self._load_hf_weights(path)
        self.actor_module = Qwen2Model(mcfg, self.store)
        # model.use_fused_kernels reaches the actor and ref configs (fsdp_workers.py:581, :658): A21 fused
        # lm_head + log-prob + entropy (csrc/fused_linear.hip) instead of logits + K2
        fused = bool(cfg.model.get("use_fused_kernels", False)) and dtype == torch.bfloat16
        cfg.actor.use_fused_kernels = fused
        cfg.ref.use_fused_kernels = fused
        # model.use_remove_padding likewise (fsdp_workers.py sets actor / ref use_remove_padding from the model)
        cfg.actor.use_remove_padding = cfg.ref.use_remove_padding = bool(cfg.model.get("use_remove_padding", False))
        # model.share_prompt_prefix (this repository's): the samples of one prompt run its tokens once in the actor /
        # ref passes (qwen2.PrefixShare; the rollout's counterpart is rollout.enable_prefix_caching)
        cfg.actor.share_prompt_prefix = cfg.ref.share_prompt_prefix = bool(cfg.model.get("share_prompt_prefix", True))
        if self._is_actor:
            o = cfg.actor.optim
            betas = tuple(o.get("betas", (0.9, 0.999)))
            self.actor_optimizer = FlatAdamW(self.store, lr=o.lr, betas=betas, eps=o.get("eps", 1e-8),
                                             weight_decay=o.weight_decay, max_grad_norm=cfg.actor.grad_clip,
                                             lr_lambda=lr_schedule(o))
            self.actor = DataParallelPPOActor(cfg.actor, self.actor_module, self.actor_optimizer)
        if self._is_rollout:
            self.rollout = MI355XRollout(self.actor_module, cfg.rollout, dp_rank=self.dp_rank)
        if self._is_ref:
            # reference policy: frozen compute-dtype copy of the initial weights (fsdp_workers.py:648-672)
            self.ref_store = ParamStore(mcfg, self.device, compute_dtype=dtype, trainable=False)
            self.ref_store.copy_from(self.store)
            self.ref_module = Qwen2Model(mcfg, self.ref_store)
            self.ref_policy = DataParallelPPOActor(cfg.ref, self.ref_module)
            if self._is_actor:  # the update's activation plan leaves room for the reference policy's store
                self.actor.extra_resident_bytes = self.ref_store.memory_bytes()

    def _load_hf_weights(self, path):
        from safetensors.torch import load_file

        sd = {}
        for f in sorted(os.listdir(path)):
            if f.endswith(".safetensors"):
                sd.update(load_file(os.path.join(path, f)))
        self.store.load_state_dict_hf(sd)

    def _out(self, d: DataProto):
        return d.to(self.output_device) if self.output_device != "cuda" else d

    # ------------------------------------------------------------------------------------------ hot path
    @register(dispatch_mode=make_nd_compute_dataproto_dispatch_fn(mesh_name="rollout"))
    @DistProfiler.annotate(color="red", role="rollout_generate")
    def generate_sequences(self, prompts: DataProto):
        """fsdp_workers.py:727-763."""
        prompts = prompts.to(self.device)
        t0 = time.perf_counter()
        output = self.rollout.generate_sequences(prompts)
        torch.cuda.synchronize()
        output.meta_info["timing"] = {"generate_sequences": time.perf_counter() - t0,
                                      "generate_prefill": getattr(self.rollout, "last_prefill_s", 0.0),
                                      "generate_capture": getattr(self.rollout, "last_capture_s", 0.0)}
        return self._out(output)

    @register(dispatch_mode=make_nd_compute_dataproto_dispatch_fn(mesh_name="actor"))
    @DistProfiler.annotate(color="blue", role="actor_compute_log_prob")
    def compute_log_prob(self, data: DataProto):
        """fsdp_workers.py:765-805: old log-probs AND entropy (calculate_entropy=True, :788)."""
        data = data.to(self.device)
        r = self.config.rollout
        data.meta_info["micro_batch_size"] = r.log_prob_micro_batch_size_per_gpu
        data.meta_info["use_dynamic_bsz"] = r.log_prob_use_dynamic_bsz
        data.meta_info["max_token_len"] = r.get("log_prob_max_token_len_per_gpu", 16384)
        data.meta_info["temperature"] = r.temperature
        output, entropys = self.actor.compute_log_prob(data=data, calculate_entropy=True)
        out = DataProto.from_dict(tensors={"old_log_probs": output, "entropys": entropys},
                                  meta_info={"temperature": r.temperature})
        return self._out(out)

    @register(dispatch_mode=make_nd_compute_dataproto_dispatch_fn(mesh_name="actor"))
    @DistProfiler.annotate(color="olive", role="ref_compute_log_prob")
    def compute_ref_log_prob(self, data: DataProto):
        """fsdp_workers.py:807-842."""
        data = data.to(self.device)
        rf = self.config.ref
        data.meta_info["micro_batch_size"] = rf.log_prob_micro_batch_size_per_gpu
        data.meta_info["temperature"] = self.config.rollout.temperature
        data.meta_info["use_dynamic_bsz"] = rf.log_prob_use_dynamic_bsz
        data.meta_info["max_token_len"] = rf.get("log_prob_max_token_len_per_gpu", 16384)
        output, _ = self.ref_policy.compute_log_prob(data=data, calculate_entropy=False)
        return self._out(DataProto.from_dict(tensors={"ref_log_prob": output}))

    @register(dispatch_mode=make_nd_compute_dataproto_dispatch_fn(mesh_name="actor"))
    @DistProfiler.annotate(color="red", role="actor_update")
    def update_actor(self, data: DataProto):
        """fsdp_workers.py:684-725 (+ MFU with an MI355X peak, lr schedule step)."""
        data = data.to(self.device)
        st = self.actor.exec_stats
        for k in st:
            st[k] = 0
        t0 = time.perf_counter()
        metrics = self.actor.update_policy(data=data)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        ntok = data.meta_info.get("global_token_num")
        if ntok:  # fsdp_workers.py:697-701
            est, promised = self.flops_counter.estimate_flops(ntok, dt)
            metrics["perf/mfu/actor"] = est * self.config.actor.ppo_epochs / promised / self.dp_size
            # what ran: the reference formula counts every row's prompt, with prompt groups run once (prefix sharing)
            # the executed forward + backward FLOPs of this rank are fewer (flops_counter.executed_flops)
            metrics["perf/mfu/actor_executed"] = self.flops_counter.executed_flops(**st) / dt / promised
        metrics["perf/max_memory_allocated_gb"] = torch.cuda.max_memory_allocated() / 1024**3
        metrics["perf/max_memory_reserved_gb"] = torch.cuda.max_memory_reserved() / 1024**3
        metrics["perf/cpu_memory_used_gb"] = psutil.virtual_memory().used / 1024**3
        metrics["actor/lr"] = self.actor_optimizer.current_lr()
        self.actor_optimizer.sched_step += 1
        return DataProto(meta_info={"metrics": metrics})

    # ------------------------------------------------------------------------------------------ checkpoint
    @register(dispatch_mode=Dispatch.ONE_TO_ALL)
    def save_checkpoint(self, local_path, hdfs_path=None, global_step=0, max_ckpt_to_keep=None):
        """fsdp_workers.py:844-880: model + optimizer + rng state (one file, or one shard file per rank)."""
        _save_store(self.store, self.actor_optimizer, local_path, "model_optim_rng",
                    {"global_step": global_step, "cuda_rng": torch.cuda.get_rng_state(),
                     "rollout_calls": self.rollout.calls if self._is_rollout else 0}, self.dp_rank)

    @register(dispatch_mode=Dispatch.ONE_TO_ALL)
    def load_checkpoint(self, local_path, hdfs_path=None, del_local_after_load=False):
        sd = _load_store(self.store, self.actor_optimizer, local_path, "model_optim_rng")
        if self._is_rollout:
            self.rollout.calls = int(sd.get("rollout_calls", 0))

    # ------------------------------------------------------------------------------------------ profiling
    @register(dispatch_mode=Dispatch.ONE_TO_ALL)
    def start_profile(self, **kwargs) -> None:
        """fsdp_workers.py:913-916 (profile.py:234-237): start profiling this rank for the current training step."""
        self.profiler.start(**kwargs)

    @register(dispatch_mode=Dispatch.ONE_TO_ALL)
    def stop_profile(self) -> None:
        """fsdp_workers.py:918-921: stop profiling this rank (tool torch: write its trace)."""
        self.profiler.stop()


def _shard_spec(section, mcfg, dp_rank, dp_size):
    """(rank, world) to shard the fp32 master + AdamW moments over (ParamStore(shard=...)), or None.
    ``fsdp_config.shard``: True / False, or "auto" = shard when DP > 1 and the replicated fp32 master +
    gradient + moments (16 B/param) would take more than 64 GB per GPU (configs #4 / #5: 7-8 B params)."""
    fc = section.get("fsdp_config", {}) or {}
    mode = fc.get("shard", "auto")
    if dp_size <= 1 or mode is False or mode == "false":
        return None
    if mode == "auto":
        n = sum(math.prod(shape) for _, shape, _ in param_specs(mcfg))
        if 16 * n <= 64 * 1024**3:
            return None
    return (dp_rank, dp_size)


# Flat-buffer layout of a checkpoint's 'master' / moment tensors. 2: the fp32 'small' region (norm weights) first,
# then the GEMM parameters in param_specs order, 64-element alignment (ParamStore); 1 (unversioned files): the
# parameters interleaved in param_specs order — loading one into a version-2 store would permute weights.
CKPT_LAYOUT_VERSION = 2


def _layout_signature(store):
    """What a checkpoint's flat tensors must agree on to be copied into ``store`` element for element."""
    return {"layout_version": CKPT_LAYOUT_VERSION, "n_small": store.n_small, "world": store.world,
            "rank": store.rank, "numel": store.numel, "master_numel": store.master.numel(),
            "offsets": [[n, int(o)] for n, (o, _, _) in store.offsets.items()]}


def _save_store(store, optim, path_dir, name, extra, dp_rank):
    """Replicated store: rank 0 writes one file. Sharded: every rank writes its shard (the reference's
    FSDP sharded checkpoint: model_world_size_{w}_rank_{r}.pt, fsdp_checkpoint_manager.py)."""
    payload = dict(extra)
    payload.update({"master": store.master.cpu(), "layout": _layout_signature(store),
                    "optim": {k: (v.cpu() if torch.is_tensor(v) else v) for k, v in optim.state_dict().items()}})
    if store.sharded:
        os.makedirs(path_dir, exist_ok=True)
        torch.save(payload, os.path.join(path_dir, f"{name}_world_size_{store.world}_rank_{store.rank}.pt"))
    elif dp_rank == 0:
        os.makedirs(path_dir, exist_ok=True)
        torch.save(payload, os.path.join(path_dir, f"{name}.pt"))
    if dist.is_initialized():
        dist.barrier()


def _load_store(store, optim, path_dir, name):
    f = (f"{name}_world_size_{store.world}_rank_{store.rank}.pt" if store.sharded else f"{name}.pt")
    sd = torch.load(os.path.join(path_dir, f), map_location="cpu", weights_only=True)
    want = _layout_signature(store)
    got = sd.get("layout")
    if got is None:
        raise ValueError(f"{f}: checkpoint without a layout record (written before layout version "
                         f"{CKPT_LAYOUT_VERSION}); its flat buffers would load permuted into this store")
    bad = [k for k in want if got.get(k) != want[k]]
    if bad:
        raise ValueError(f"{f}: flat-buffer layout differs from this store in {bad} "
                         f"(checkpoint layout_version {got.get('layout_version')}, store {CKPT_LAYOUT_VERSION})")
    if sd["master"].shape != store.master.shape or sd["optim"]["exp_avg"].shape != optim.exp_avg.shape:
        raise ValueError(f"{f}: buffer shapes {tuple(sd['master'].shape)} do not match {tuple(store.master.shape)}")
    store.master.copy_(sd["master"])
    store.refresh_compute()
    optim.load_state_dict(sd["optim"])
    return sd


class CriticWorker(Worker):
    """fsdp_workers.py:922-1340 for ``critic.strategy = "mi355x"``: Qwen2 backbone + `score` value head
    (num_labels=1, classifier dropout 0), replicated-parameter DP with one RCCL all-reduce per optimizer step."""

    def __init__(self, config, output_device: str = "cuda"):
        super().__init__()
        self.config = config
        self.output_device = output_device
        self.device = torch.device("cuda", torch.cuda.current_device())
        dp = dist.get_world_size() if dist.is_initialized() else 1
        self.dp_size = dp
        self.dp_rank = dist.get_rank() if dist.is_initialized() else 0
        self._register_dispatch_collect_info("critic", dp_rank=self.dp_rank, is_collect=True)
        self.profiler = DistProfiler(rank=self.dp_rank, config=config.get("profiler"))  # fsdp_workers.py:927-937
        # fsdp_workers.py:979-1000 batch-size normalisation
        c = config
        c.ppo_mini_batch_size = c.ppo_mini_batch_size * c.get("rollout_n", 1) // dp
        if c.get("ppo_micro_batch_size") is not None:
            c.ppo_micro_batch_size_per_gpu = c.ppo_micro_batch_size // dp
            c.forward_micro_batch_size_per_gpu = c.get("forward_micro_batch_size", c.ppo_micro_batch_size) // dp
        if c.get("forward_micro_batch_size_per_gpu") is None:
            c.forward_micro_batch_size_per_gpu = c.ppo_micro_batch_size_per_gpu
        if c.get("ppo_micro_batch_size_per_gpu") is not None:
            assert c.ppo_mini_batch_size % c.ppo_micro_batch_size_per_gpu == 0, (
                f"normalized ppo_mini_batch_size {c.ppo_mini_batch_size} should be divisible by "
                f"ppo_micro_batch_size_per_gpu {c.ppo_micro_batch_size_per_gpu}")

    @register(dispatch_mode=Dispatch.ONE_TO_ALL)
    def init_model(self):
        """fsdp_workers.py:1003-1123 (_build_critic_model_optimizer + DataParallelPPOCritic)."""
        cfg = self.config
        mcfg = resolve_model_config(cfg.model)
        mcfg.num_labels = 1
        self.model_config = mcfg
        self.flops_counter = FlopsCounter(mcfg)
        dtype = torch.float32 if cfg.model.get("dtype", "bfloat16") == "float32" else torch.bfloat16
        shard = _shard_spec(cfg, mcfg, self.dp_rank, self.dp_size)
        self.store = ParamStore(mcfg, self.device, compute_dtype=dtype, trainable=True, shard=shard)
        path = cfg.model.get("path", "random:")
        if path.startswith("random:"):
            self.store.init_random(int(cfg.model.get("seed", 4321)))
        else:
            from safetensors.torch import load_file

            sd = {}
            for f in sorted(os.listdir(path)):
                if f.endswith(".safetensors"):
                    sd.update(load_file(os.path.join(path, f)))
            self.store.load_state_dict_hf(sd)
        self.critic_module = Qwen2Model(mcfg, self.store)
        o = cfg.optim
        self.critic_optimizer = FlatAdamW(self.store, lr=o.lr, betas=tuple(o.get("betas", (0.9, 0.999))),
                                          eps=o.get("eps", 1e-8), weight_decay=o.weight_decay,
                                          max_grad_norm=cfg.grad_clip, lr_lambda=lr_schedule(o))
        self.critic = DataParallelPPOCritic(cfg, self.critic_module, self.critic_optimizer)

    def _out(self, d: DataProto):
        return d.to(self.output_device) if self.output_device != "cuda" else d

    @register(dispatch_mode=make_nd_compute_dataproto_dispatch_fn(mesh_name="critic"))
    @DistProfiler.annotate(color="cyan")
    def compute_values(self, data: DataProto):
        """fsdp_workers.py:1237-1258 -> values (bs, R) in the compute dtype."""
        data = data.to(self.device)
        data.meta_info["micro_batch_size"] = self.config.forward_micro_batch_size_per_gpu
        data.meta_info["max_token_len"] = self.config.get("forward_max_token_len_per_gpu", 32768)
        data.meta_info["use_dynamic_bsz"] = self.config.get("use_dynamic_bsz", False)
        values = self.critic.compute_values(data=data)
        return self._out(DataProto.from_dict(tensors={"values": values}))

    @register(dispatch_mode=make_nd_compute_dataproto_dispatch_fn(mesh_name="critic"))
    @DistProfiler.annotate(color="pink")
    def update_critic(self, data: DataProto):
        """fsdp_workers.py:1260-1292 (+ perf/mfu/critic with the MI355X peak, critic/lr, lr schedule step)."""
        data = data.to(self.device)
        t0 = time.perf_counter()
        metrics = self.critic.update_critic(data=data)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        ntok = data.meta_info.get("global_token_num")
        if ntok:  # fsdp_workers.py:1275-1279
            est, promised = self.flops_counter.estimate_flops(ntok, dt)
            metrics["perf/mfu/critic"] = est * self.config.ppo_epochs / promised / self.dp_size
        metrics["critic/lr"] = self.critic_optimizer.current_lr()
        self.critic_optimizer.sched_step += 1
        return DataProto(meta_info={"metrics": metrics})

    @register(dispatch_mode=Dispatch.ONE_TO_ALL)
    def save_checkpoint(self, local_path, hdfs_path=None, global_step=0, max_ckpt_to_keep=None):
        """fsdp_workers.py:1294-1310: model + optimizer (one file, or one shard file per rank)."""
        _save_store(self.store, self.critic_optimizer, local_path, "critic_model_optim", {"global_step": global_step},
                    self.dp_rank)

    @register(dispatch_mode=Dispatch.ONE_TO_ALL)
    def load_checkpoint(self, local_path, hdfs_path=None, del_local_after_load=True):
        _load_store(self.store, self.critic_optimizer, local_path, "critic_model_optim")

    # ------------------------------------------------------------------------------------------ profiling
    @register(dispatch_mode=Dispatch.ONE_TO_ALL)
    def start_profile(self, **kwargs) -> None:
        """fsdp_workers.py:913-916 (profile.py:234-237): start profiling this rank for the current training step."""
        self.profiler.start(**kwargs)

    @register(dispatch_mode=Dispatch.ONE_TO_ALL)
    def stop_profile(self) -> None:
        """fsdp_workers.py:918-921: stop profiling this rank (tool torch: write its trace)."""
        self.profiler.stop()
