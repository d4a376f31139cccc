"""Worker profiling for the hot path: verl/utils/profiler (DistProfiler, DistProfilerExtension, annotate) on MI355X.

The reference gives every worker a ``DistProfiler`` (``fsdp_workers.py:168-196``), registers
``start_profile(**kwargs)`` / ``stop_profile()`` ONE_TO_ALL (``profile.py:220-243``, ``fsdp_workers.py:913-921``)
which the trainer calls around the steps listed in ``global_profiler.steps`` (``ray_trainer.py:1011-1031,
1096-1113, 1355-1366``), and marks the four hot methods with ``@DistProfiler.annotate`` (``fsdp_workers.py:685, 728,
766, 808``; critic ``:1238, :1260``) — NVTX ranges for Nsight Systems in its CUDA build (``nvtx_profile.py:113-200``).

Here the tools are the ROCm ones:

* ``tool: roctx`` — each annotated method is one roctx range (``roctxRangePushA`` / ``roctxRangePop`` of
  rocprofiler-sdk's roctx library, the marker API ``rocprofv3 --marker-trace`` records next to its kernel trace),
  pushed only inside a started profile (``start_profile`` .. ``stop_profile``), as the reference's nsys ranges are.
* ``tool: torch`` — ``torch.profiler`` over CPU + the HIP device between ``start_profile`` and ``stop_profile``
  (``profile.py:24-121``), the ranges as ``record_function`` spans, and a Chrome trace written at ``stop_profile``
  to ``{save_path}/prof_step_{step}_rank_{rank}.json``.

Config (the reference's ``ProfilerConfig`` keys, ``profiler/config.py:89-125``): ``tool``, ``enable``, ``all_ranks``,
``ranks``, ``save_path``; ``tool_config.torch.step_start`` / ``step_end`` are accepted and unused (the trainer's
``global_profiler.steps`` decides which steps run between start and stop, as with nsys).
"""

from __future__ import annotations

import ctypes
import functools
import os
from typing import Callable, Optional

import torch

TOOLS = (None, "roctx", "torch")

_ROCTX = None


def _roctx():
    """rocprofiler-sdk's roctx (the library rocprofv3's marker tracing intercepts); torch's nvtx shim (roctracer's
    roctx on a ROCm build of torch) when that is absent. Loaded on first use."""
    global _ROCTX
    if _ROCTX is None:
        lib = None
        roots = [os.environ.get("ROCM_PATH", "/opt/rocm"), "/opt/rocm"]
        for root in roots:
            for name in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so"):
                try:
                    lib = ctypes.CDLL(os.path.join(root, "lib", name))
                    break
                except OSError:
                    continue
            if lib is not None:
                break
        if lib is not None:
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.argtypes = []
            lib.roctxRangePop.restype = ctypes.c_int
            _ROCTX = (lambda s: lib.roctxRangePushA(s.encode()), lib.roctxRangePop)
        else:
            _ROCTX = (torch.cuda.nvtx.range_push, torch.cuda.nvtx.range_pop)
    return _ROCTX


def mark_start_range(message: Optional[str] = None, color: Optional[str] = None, domain: Optional[str] = None,
                     category: Optional[str] = None):
    """nvtx_profile.py:31-56 — push a roctx range; returns the handle mark_end_range pops."""
    push, _ = _roctx()
    push(message or "range")
    return message


def mark_end_range(range_id) -> None:
    _, pop = _roctx()
    pop()


def _get(cfg, key, default=None):
    if cfg is None:
        return default
    if isinstance(cfg, dict):
        return cfg.get(key, default)
    return getattr(cfg, key, default)


class DistProfiler:
    """profile.py:174-216 / nvtx_profile.py:113-200 with roctx and torch.profiler as the tools."""

    def __init__(self, rank: int, config=None, **kwargs):
        tool = _get(config, "tool")
        self.enable = bool(_get(config, "enable", False)) and tool is not None
        if tool not in TOOLS:
            raise ValueError(f"profiler tool {tool!r}: this backend profiles with {TOOLS[1:]} (rocprofv3 / torch)")
        self.tool = tool
        self.rank = rank
        self.this_step = False
        ranks = _get(config, "ranks", None) or []
        self.this_rank = self.enable and (bool(_get(config, "all_ranks", False)) or rank in list(ranks))
        self.save_path = _get(config, "save_path", None) or "outputs/profile"
        self.discrete = bool(_get(_get(_get(config, "tool_config"), "roctx"), "discrete", False))
        self.prof = None
        self.step = None
        self.traces = []  # files written by stop() (tool torch)

    def start(self, **kwargs):
        """Start profiling this rank for the current training step (``role`` / ``profile_step`` as the trainer passes
        them, ray_trainer.py:1014)."""
        if not (self.enable and self.this_rank):
            return
        self.this_step = True
        self.step = kwargs.get("profile_step", self.step)
        if self.tool == "torch":
            acts = [torch.profiler.ProfilerActivity.CPU]
            if torch.cuda.is_available():
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            self.prof = torch.profiler.profile(activities=acts, record_shapes=False, with_stack=False)
            self.prof.start()

    def stop(self):
        if not (self.enable and self.this_rank) or not self.this_step:
            return
        self.this_step = False
        if self.tool == "torch" and self.prof is not None:
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            self.prof.stop()
            os.makedirs(self.save_path, exist_ok=True)
            step = self.step if self.step is not None else len(self.traces)
            path = os.path.join(self.save_path, f"prof_step_{step}_rank_{self.rank}.json")
            self.prof.export_chrome_trace(path)
            self.traces.append(path)
            self.prof = None

    @staticmethod
    def annotate(message: Optional[str] = None, color: Optional[str] = None, domain: Optional[str] = None,
                 category: Optional[str] = None, **kwargs) -> Callable:
        """Decorate a worker method (a ``self.profiler`` DistProfiler) with one range named ``message`` or the method's
        name, recorded only while a profile of this rank is started (nvtx_profile.py:161-200)."""

        def decorator(func):
            @functools.wraps(func)
            def wrapper(self, *args, **kw):
                prof = getattr(self, "profiler", None)
                if prof is None or not prof.enable or not prof.this_step:
                    return func(self, *args, **kw)
                name = message or func.__name__
                if prof.tool == "torch":
                    with torch.profiler.record_function(name):
                        return func(self, *args, **kw)
                mark_start_range(message=name, color=color, domain=domain, category=category)
                try:
                    return func(self, *args, **kw)
                finally:
                    mark_end_range(name)

            return wrapper

        return decorator


def profiler_config(*sections):
    """The first section among ``sections`` that enables a profiler (fsdp_workers.py:168-196 picks the actor's, else
    the rollout's, else the ref's), or None."""
    for s in sections:
        p = _get(s, "profiler")
        if p is not None and _get(p, "enable", False):
            return p
    return None


__all__ = ["DistProfiler", "mark_start_range", "mark_end_range", "profiler_config", "TOOLS"]
