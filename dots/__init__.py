"""Import bridge: exposes the on-disk package directory ``dots.rl_amd/`` as the module ``dots.rl_amd``.

A directory name containing a dot cannot be imported by the normal finder, so this package maps the
submodule ``rl_amd`` onto it (``import dots.rl_amd`` / ``from dots.rl_amd import ...`` both work).
"""

import importlib.util
import os
import sys

_PKG_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dots.rl_amd")

if "dots.rl_amd" not in sys.modules:
    _spec = importlib.util.spec_from_file_location(
        "dots.rl_amd", os.path.join(_PKG_DIR, "__init__.py"), submodule_search_locations=[_PKG_DIR])
    rl_amd = importlib.util.module_from_spec(_spec)
    sys.modules["dots.rl_amd"] = rl_amd
    _spec.loader.exec_module(rl_amd)
else:
    rl_amd = sys.modules["dots.rl_amd"]
