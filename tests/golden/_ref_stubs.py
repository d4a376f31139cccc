"""Dependency stubs that let the reference's hot-path modules import in the survey container.

Used ONLY by ``tests/golden/make_golden.py`` (run here, never on the GPU box) to call the
reference implementation and record golden vectors. See SURVEY.md §8(c) for the recipe:
``ray``, ``tensordict``, ``omegaconf`` and ``codetiming`` are not installed, and the hot-path
modules only touch them at import time (plus a dict-backed TensorDict for DataProto users).
"""

import contextlib
import importlib.abc
import importlib.machinery
import sys
import types

REFERENCE_ROOT = "/root/reference"


def install():
    _auto_stub(["ray", "torchdata"])

    td = types.ModuleType("tensordict")
    td.__version__ = "0.9.1"
    td.TensorDict = _tensordict_class()
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


class _Inert:
    """Stand-in for any attribute of an auto-stubbed package: callable (a decorator returns its argument),
    subclassable, attribute access yields another inert object."""

    def __init__(self, *a, **k):
        pass

    def __call__(self, *a, **k):
        if len(a) == 1 and not k and callable(a[0]):
            return a[0]
        return _Inert()

    def __getattr__(self, k):
        if k.startswith("__"):
            raise AttributeError(k)
        return _Inert()

    def __mro_entries__(self, bases):
        return (object,)


class _AutoModule(types.ModuleType):
    def __getattr__(self, k):
        if k.startswith("__"):
            raise AttributeError(k)
        return _Inert()


class _AutoFinder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    def __init__(self, roots):
        self.roots = set(roots)

    def find_spec(self, name, path, target=None):
        if name.split(".")[0] in self.roots:
            return importlib.machinery.ModuleSpec(name, self, is_package=True)
        return None

    def create_module(self, spec):
        m = _AutoModule(spec.name)
        m.__path__ = []
        return m

    def exec_module(self, module):
        return None


def _auto_stub(roots):
    """Packages absent from the container (ray, torchdata) that the reference touches only at import time on the
    code paths the golden generators run."""
    for k in list(sys.modules):
        if k.split(".")[0] in roots:
            del sys.modules[k]
    sys.meta_path.insert(0, _AutoFinder(roots))


def _tensordict_class():
    import torch

    class TensorDict(dict):
        """Dict-backed stand-in for tensordict.TensorDict with the operations DataProto and the actor use:
        batch_size, str / int / slice / index access, select, to, chunk, pop, torch.cat."""

        def __init__(self, source=None, batch_size=None, device=None, **_):
            super().__init__(source or {})
            if batch_size is None:
                batch_size = []
            if isinstance(batch_size, int):
                batch_size = [batch_size]
            self.batch_size = torch.Size(list(batch_size))
            self.device = device

        def keys(self):
            return list(super().keys())

        def _rows(self, rows):
            n = next(iter(rows.values())).shape[0] if rows else 0
            return TensorDict(rows, batch_size=[n])

        def __getitem__(self, key):
            if isinstance(key, str):
                return super().__getitem__(key)
            rows = {k: v[key] for k, v in self.items()}
            if isinstance(key, int):
                return TensorDict(rows, batch_size=[])
            return self._rows(rows)

        def select(self, *keys):
            return TensorDict({k: super(TensorDict, self).__getitem__(k) for k in keys}, batch_size=self.batch_size)

        def to(self, device):
            return TensorDict({k: v.to(device) for k, v in self.items()}, batch_size=self.batch_size, device=device)

        def chunk(self, chunks, dim=0):
            parts = {k: torch.chunk(v, chunks, dim) for k, v in self.items()}
            n = len(next(iter(parts.values())))
            return [self._rows({k: p[i] for k, p in parts.items()}) for i in range(n)]

        def contiguous(self):
            return TensorDict({k: v.contiguous() for k, v in self.items()}, batch_size=self.batch_size)

        def consolidate(self):
            return self

        @classmethod
        def __torch_function__(cls, func, types, args=(), kwargs=None):
            kwargs = kwargs or {}
            if func is torch.cat:
                lst = args[0]
                dim = args[1] if len(args) > 1 else kwargs.get("dim", 0)
                keys = lst[0].keys()
                out = {k: torch.cat([t[k] for t in lst], dim) for k in keys}
                return TensorDict(out, batch_size=[sum(t.batch_size[0] for t in lst)])
            return NotImplemented

    return TensorDict
