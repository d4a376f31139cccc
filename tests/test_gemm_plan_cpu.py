"""drl_gemm's decomposition rules (csrc/gemm_sk.hip plan_decomposition) pinned on the CPU through drl_gemm_plan: the
pass shapes of config #2 over 256 CUs (MI355X), each rule with the measurement it came from cited in the source."""
import ctypes
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "dots.rl_amd", "libdotsrl_amd.so")

PLAIN, BIAS, SWIGLU, SWIGLU_BWD = 0, 1, 2, 3
CUS = 256


@pytest.fixture(scope="module")
def plan():
    from dots.rl_amd import _lib

    if not os.path.exists(LIB):
        subprocess.run(["make", "-C", os.path.join(ROOT, "dots.rl_amd", "csrc"), "-j8"], check=True)
    lib = _lib.load(LIB)
    lib.drl_gemm_set_sk_tuning(0, 0, 0, 0)

    def f(M, N, K, epi=PLAIN):
        info = (ctypes.c_int32 * 5)()
        assert lib.drl_gemm_plan(M, N, K, epi, CUS, info) == 0
        return dict(mode=info[0], splits=info[1], grid=info[2], dp_tiles=info[3], sk_base=info[4])

    return f


def test_small_weight_gradients_take_uniform_split_k(plan):
    # qkv / o weight gradients over the update pass's 82144 tokens: 20 / 16 tiles x 642 k-pairs
    assert plan(1152, 896, 82144) == dict(mode=3, splits=12, grid=240, dp_tiles=0, sk_base=0)
    assert plan(896, 896, 82144) == dict(mode=3, splits=16, grid=256, dp_tiles=0, sk_base=0)


@pytest.mark.parametrize("T", [82144, 164288])
def test_down_weight_gradient_three_slices(plan, T):
    # 76 tiles x 642 / 1284 k-pairs: 3 uniform split-K slices (not stream-K)
    assert plan(896, 4864, T) == dict(mode=3, splits=3, grid=228, dp_tiles=0, sk_base=0)


def test_few_tiles_over_very_long_k_stay_on_stream_k(plan):
    # the lm_head input gradient at 7000 / 8192 rows: 112 / 128 tiles x 1187 k-pairs
    assert plan(7000, 896, 151936)["mode"] == 1
    assert plan(8192, 896, 151936)["mode"] == 1


@pytest.mark.parametrize("M", [82144, 164288])
def test_swiglu_forward_over_many_rounds_is_persistent_stream_k(plan, M):
    p = plan(M, 9728, 896, SWIGLU)
    assert p["mode"] == 1 and p["grid"] == CUS


def test_short_swiglu_forward_stays_on_whole_tiles(plan):
    assert plan(6144, 9728, 896, SWIGLU) == dict(mode=2, splits=1, grid=24 * 38, dp_tiles=24 * 38, sk_base=0)


def test_tail_split_k(plan):
    # down_proj forward at 82144 rows: 1284 tiles = 5 x 256 + 4, 38 k-pairs: the last 4 tiles over 16 slices
    assert plan(82144, 896, 4864) == dict(mode=2, splits=16, grid=1280 + 64, dp_tiles=1280, sk_base=1280)
    # the lm_head weight gradient's K blocks: 2376 tiles = 9 x 256 + 72 (a third of the CUs), 52 k-pairs: 3 slices
    assert plan(151936, 896, 6656) == dict(mode=2, splits=3, grid=2304 + 216, dp_tiles=2304, sk_base=2304)
    # K = 896 (7 k-pairs): no tail split (its fill and combine cost more than the round)
    assert plan(82144, 896, 896) == dict(mode=2, splits=1, grid=1284, dp_tiles=1284, sk_base=0)
    # whole-tile epilogues never split
    assert plan(82144, 4864, 896, SWIGLU_BWD)["splits"] == 1


@pytest.mark.parametrize("T", [82144, 164288, 98304, 196608])
def test_concurrent_pairs_never_pair_two_spinning_plans(plan, T):
    """Co-residency rule (c) of the gemm_sk.hip header: qwen2.dgrad_wgrad runs a weight gradient beside its input
    gradient only where the weight gradient's whole tiles leave CUs idle (qwen2._concurrent_pair), and at most one of
    the pair may spin-wait. Config #2's projections at the update pass's token counts: gate_up (the only concurrent
    pair) has a non-spinning weight gradient beside a tail-split input gradient."""

    def spins(p):
        return p["mode"] in (1, 3) or p["splits"] > 1

    H, I, NQ, HD = 896, 4864, 1152, 896
    for out, inp in ((NQ, H), (H, HD), (2 * I, H), (H, I)):
        tiles = -(-out // 256) * -(-inp // 256)
        if not (CUS < 2 * tiles and tiles < CUS):  # qwen2._concurrent_pair
            continue
        wgrad, dgrad = plan(out, inp, T), plan(T, inp, out)
        assert not (spins(wgrad) and spins(dgrad)), (out, inp, T, wgrad, dgrad)
    # the measurement switch DRL_CONCURRENT_DOWN pairs down_proj's split-K weight gradient with the whole-tile
    # SwiGLU-backward input gradient
    assert not spins(plan(T, I, H, SWIGLU_BWD))


def test_native_gemm_spins_matches_the_plan():
    from dots.rl_amd import native

    assert native.gemm_spins(82144, 896, 4864, cus=CUS)          # tail split-K
    assert not native.gemm_spins(82144, 896, 896, cus=CUS)       # whole tiles
    assert native.gemm_spins(896, 896, 82144, cus=CUS)           # uniform split-K
    assert not native.gemm_spins(9728, 896, 82144, cus=CUS)      # gate_up weight gradient: whole tiles
