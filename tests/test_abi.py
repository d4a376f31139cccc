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
    assert lib.drl_abi_version() == 2


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
