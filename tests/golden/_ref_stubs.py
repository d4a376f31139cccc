"""Dependency stubs that let the reference's hot-path modules import in the survey container.

Used ONLY by ``tests/golden/make_golden.py`` (run here, never on the GPU box) to call the
reference implementation and record golden vectors. See SURVEY.md §8(c) for the recipe:
``ray``, ``tensordict``, ``omegaconf`` and ``codetiming`` are not installed, and the hot-path
modules only touch them at import time (plus a dict-backed TensorDict for DataProto users).
"""

import contextlib
import sys
import types

REFERENCE_ROOT = "/root/reference"


def install():
    ray = types.ModuleType("ray")
    ray.ObjectRef = type("ObjectRef", (), {})
    ray.remote = lambda *a, **k: (a[0] if a and callable(a[0]) else (lambda f: f))
    for name in ["ray", "ray.util", "ray.actor", "ray.util.placement_group", "ray.util.scheduling_strategies"]:
        sys.modules[name] = ray if name == "ray" else types.ModuleType(name)

    td = types.ModuleType("tensordict")
    td.__version__ = "0.9.1"

    class TensorDict(dict):
        """Dict-backed stand-in: enough for code that only indexes tensors by key."""

        def __init__(self, source=None, batch_size=None, **_):
            super().__init__(source or {})
            self.batch_size = [batch_size] if isinstance(batch_size, int) else list(batch_size or [])

        def keys(self):
            return list(super().keys())

        def __getitem__(self, key):  # str -> tensor; int / slice / index -> the rows (DataProtoItem access)
            if isinstance(key, str):
                return super().__getitem__(key)
            rows = {k: v[key] for k, v in self.items()}
            n = next(iter(rows.values())).shape[:1] if rows and not isinstance(key, int) else []
            return TensorDict(rows, batch_size=list(n))

    td.TensorDict = TensorDict
    sys.modules["tensordict"] = td

    oc = types.ModuleType("omegaconf")

    class DictConfig(dict):
        def __getattr__(self, k):
            try:
                return self[k]
            except KeyError as e:
                raise AttributeError(k) from e

    class ListConfig(list):
        pass

    class OmegaConf:
        @staticmethod
        def is_config(x):
            return isinstance(x, (DictConfig, ListConfig))

        @staticmethod
        def to_container(x, resolve=True):
            return x

        @staticmethod
        def create(x):
            return DictConfig(x)

        @staticmethod
        def set_struct(*_a, **_k):
            return None

    oc.DictConfig = DictConfig
    oc.ListConfig = ListConfig
    oc.MISSING = "???"
    oc.OmegaConf = OmegaConf
    oc.open_dict = lambda *_a, **_k: contextlib.nullcontext()
    sys.modules["omegaconf"] = oc

    ct = types.ModuleType("codetiming")

    class Timer:
        def __init__(self, *a, **k):
            self.last = 0.0

        def __enter__(self):
            return self

        def __exit__(self, *a):
            return False

    ct.Timer = Timer
    sys.modules["codetiming"] = ct
    if REFERENCE_ROOT not in sys.path:
        sys.path.insert(0, REFERENCE_ROOT)
    return DictConfig
