"""Single-controller mechanics: ``Worker``, ``@register`` + ``Dispatch``, and an SPMD ``WorkerGroup``.

Mirrors verl/single_controller/base/{decorator.py,worker.py,worker_group.py}: worker methods are plain
methods decorated with a dispatch mode; a WorkerGroup binds them so the driver calls
``wg.compute_log_prob(batch)`` and gets the whole batch's result back.

MI355X-first process model: one process per GPU launched by ``torch.distributed.run`` (no Ray). The
driver logic runs SPMD on every rank; "dispatch" is taking this rank's chunk of the (replicated)
DataProto and "collect" is an all-gather of the rank outputs over RCCL (device tensors) — the
equivalent of decorator.py:213-312's chunk / ray.put / concat, with no pickling of tensors.
"""

from __future__ import annotations

import functools
import os
from enum import Enum

import torch
import torch.distributed as dist

from .protocol import DataProto

MAGIC_ATTR = "attrs_3141562937"  # same attribute name the reference decorator uses


class Dispatch(Enum):
    RANK_ZERO = 0
    ONE_TO_ALL = 1
    ALL_TO_ALL = 2
    DP_COMPUTE = 3
    DP_COMPUTE_PROTO = 4
    DP_COMPUTE_PROTO_WITH_FUNC = 5
    DP_COMPUTE_METRIC = 6
    DIRECT_ROLLOUT_METHOD = 7


class Execute(Enum):
    ALL = 0
    RANK_ZERO = 1


def make_nd_compute_dataproto_dispatch_fn(mesh_name):
    """decorator.py:213-312 — DP dispatch over the named mesh. With one DP mesh per process group this is
    DP_COMPUTE_PROTO; the mesh name is kept for the worker's dispatch-info registry."""
    return {"mesh_name": mesh_name, "mode": Dispatch.DP_COMPUTE_PROTO}


def register(dispatch_mode=Dispatch.ALL_TO_ALL, execute_mode=Execute.ALL, blocking=True, materialize_futures=True):
    """decorator.py:410-452 — tag a worker method with its dispatch/collect contract."""

    def decorator(func):
        @functools.wraps(func)
        def inner(*args, **kwargs):
            return func(*args, **kwargs)

        setattr(inner, MAGIC_ATTR, {"dispatch_mode": dispatch_mode, "execute_mode": execute_mode,
                                    "blocking": blocking})
        return inner

    return decorator


class Worker:
    """worker.py:72-308 — rank / world wiring from the launcher environment."""

    def __init__(self):
        self._rank = int(os.environ.get("RANK", "0"))
        self._world_size = int(os.environ.get("WORLD_SIZE", "1"))
        self._local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.__dispatch_dp_rank = {}
        self.__collect_dp_rank = {}

    @property
    def rank(self):
        return self._rank

    @property
    def world_size(self):
        return self._world_size

    def _register_dispatch_collect_info(self, mesh_name: str, dp_rank: int, is_collect: bool):
        self.__dispatch_dp_rank[mesh_name] = dp_rank
        self.__collect_dp_rank[mesh_name] = is_collect

    def _query_dispatch_info(self, mesh_name: str):
        return self.__dispatch_dp_rank.get(mesh_name, self._rank)

    def _query_collect_info(self, mesh_name: str):
        return self.__collect_dp_rank.get(mesh_name, True)


class SPMDWorkerGroup:
    """WorkerGroup over the process group: every rank holds one local worker and runs the driver SPMD.

    Bound methods follow the decorated dispatch mode:
      ONE_TO_ALL / ALL_TO_ALL   -> call the local worker with the same arguments (returns [result])
      DP_COMPUTE_PROTO (+ nd)   -> DataProto.chunk(dp_size)[dp_rank] -> method -> all-gather of the outputs
      RANK_ZERO                 -> only rank 0 runs it
    """

    def __init__(self, worker: Worker, group=None):
        self.worker = worker
        self.group = group
        self.world_size = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self._bind_worker_methods()

    def _bind_worker_methods(self):
        for name in dir(type(self.worker)):
            fn = getattr(type(self.worker), name, None)
            attrs = getattr(fn, MAGIC_ATTR, None)
            if attrs is None:
                continue
            setattr(self, name, self._make_caller(name, attrs))

    def _make_caller(self, name, attrs):
        mode = attrs["dispatch_mode"]
        mesh = None
        if isinstance(mode, dict):
            mesh, mode = mode["mesh_name"], mode["mode"]
        method = getattr(self.worker, name)

        def call(*args, **kwargs):
            if mode in (Dispatch.ONE_TO_ALL, Dispatch.ALL_TO_ALL):
                return [method(*args, **kwargs)]
            if mode == Dispatch.RANK_ZERO:
                return method(*args, **kwargs) if self.rank == 0 else None
            if mode in (Dispatch.DP_COMPUTE_PROTO, Dispatch.DP_COMPUTE):
                dp_rank = self.worker._query_dispatch_info(mesh) if mesh else self.rank
                args = [a.chunk(self.world_size)[dp_rank] if isinstance(a, DataProto) else a for a in args]
                kwargs = {k: (v.chunk(self.world_size)[dp_rank] if isinstance(v, DataProto) else v)
                          for k, v in kwargs.items()}
                out = method(*args, **kwargs)
                if isinstance(out, DataProto) and out.batch is not None and len(out.batch):
                    return out.all_gather(self.group)
                return out
            raise NotImplementedError(f"dispatch mode {mode}")

        call.__name__ = name
        return call


def init_process_group_from_env(backend: str | None = None):
    """One process per GPU (torch.distributed.run env); RCCL ('nccl') on GPU, gloo on CPU."""
    if dist.is_initialized():
        return
    if "WORLD_SIZE" not in os.environ or int(os.environ["WORLD_SIZE"]) == 1 and "MASTER_ADDR" not in os.environ:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 1000))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        os.environ.setdefault("LOCAL_RANK", "0")
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    dist.init_process_group(backend=backend)
