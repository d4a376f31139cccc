"""CPU checks of the drop-in boundary: the HIP library builds for gfx950, loads, and exports exactly the
C-ABI that include/dotsrl_amd.h declares (no compute calls: there is no GPU here)."""

import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dotsrl_amd.h")
LIB = os.path.join(ROOT, "dots.rl_amd", "libdotsrl_amd.so")


@pytest.fixture(scope="module")
def built_lib():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-C", os.path.join(ROOT, "dots.rl_amd", "csrc"), "-j8"], check=True)
    return LIB


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(drl_[a-z0-9_]+)\s*\(", src)))


def header_abi_version():
    return int(re.search(r"#define DRL_ABI_VERSION (\d+)", open(HEADER).read()).group(1))


def header_struct_fields(name):
    """Field names of `typedef struct name {...} name;` in the header, in order."""
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (name, name), src, flags=re.S).group(1)
    return re.findall(r"(\w+)\s*;", body)


def test_ppo_loss_params_layout_agrees_everywhere():
    """The K1 parameter struct: header == ctypes binding (_lib.PPOLossParams) == the binding INTEGRATION.md §3
    shows a verl maintainer (a short struct there would be read past its end by the library)."""
    from dots.rl_amd import _lib

    fields = header_struct_fields("drl_ppo_loss_params")
    assert [f for f, _ in _lib.PPOLossParams._fields_] == fields
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    block = re.search(r"class PPOLossParams\(ctypes.Structure\):(.*?)\]\n", doc, flags=re.S).group(1)
    assert re.findall(r'\("(\w+)", ctypes', block) == fields
    assert f"drl_abi_version() == {header_abi_version()}" in doc


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ["drl_ppo_loss_fwd_bwd", "drl_logprob_entropy_fwd", "drl_logprob_entropy_bwd",
                 "drl_grpo_outcome_advantage", "drl_gae_advantage_return", "drl_select_tokens", "drl_adamw_step"]:
        assert must in names


def test_library_exports_every_declared_symbol(built_lib):
    lib = ctypes.CDLL(built_lib)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", built_lib], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (drl_[a-z0-9_]+)", out))
    assert exported == set(declared_functions())


def test_python_binding_signatures_cover_the_header(built_lib):
    from dots.rl_amd import _lib

    assert set(_lib.SIGNATURES) == set(declared_functions())
    lib = _lib.load(built_lib)
    assert lib.drl_abi_version() == _lib.ABI_VERSION == header_abi_version()


def test_library_is_gfx950_code(built_lib):
    data = open(built_lib, "rb").read()
    assert b"gfx950" in data  # offload bundle id of the embedded code object
    sections = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", built_lib], capture_output=True,
                              text=True, check=True).stdout
    assert ".hip_fatbin" in sections


def test_errors_are_reported_without_a_gpu(built_lib):
    from dots.rl_amd import _lib

    lib = _lib.load(built_lib)
    prm = _lib.PPOLossParams(0.2, 0.2, 0.5, 0.0, 0.0, 1.0, 0, -1)  # clip_ratio_c <= 1 is rejected before any HIP call
    rc = lib.drl_ppo_loss_fwd_bwd(1, 1, 1, 1, 0, None, None, 2, 2, ctypes.byref(prm), 1, None, None, None, 0, None)
    assert rc == -1
    assert b"clip_ratio_c" in lib.drl_last_error()
