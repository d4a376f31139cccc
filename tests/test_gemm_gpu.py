"""Full-sequence projection GEMMs (csrc/gemm.hip) against the fp32 product of the same bf16 operands: each
output within one bf16 rounding of the fp32 reference (a different fp32 summation order can move a value that
lies near a rounding boundary by one bf16 ulp); the SwiGLU epilogue against swiglu_fwd on the reference
pre-activation; bias with addmm's single rounding; ragged M / N tails; deterministic."""

import pytest
import torch

from dots.rl_amd import native

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16


@pytest.fixture(params=[0, 9], ids=["auto", "pingpong"], autouse=True)
def tile(request):
    """every test under the automatic tile choice and under the 256 x 256 ping-pong form (tile 9)"""
    native.lib().drl_gemm_set_tile(request.param)
    yield request.param
    native.lib().drl_gemm_set_tile(0)


def rnd(*shape, scale=1.0, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return (torch.randn(*shape, device=DEV, generator=g) * scale).to(BF)


def _check_bf16(got, ref):
    """got (bf16) within one bf16 ulp of the fp32 reference, almost everywhere exactly its rounding."""
    ref_b = ref.to(BF).float()
    g = got.float()
    # one bf16 ulp of the value, plus the fp32 summation-order error where the sum cancels to near zero
    tol = ref.abs() * 2.0 ** -7 * 1.01 + 1e-5 * ref.abs().max()
    assert ((g - ref).abs() <= tol).all(), ((g - ref).abs() - tol).max().item()
    assert (g != ref_b).float().mean().item() < 0.02


@pytest.mark.parametrize("M,N,K", [(6144, 896, 896), (6144, 1152, 896), (12288, 896, 4864), (300, 896, 896),
                                   (1000, 200, 128), (4096, 9728, 896), (130, 64, 64)])
def test_gemm_plain(M, N, K):
    x = rnd(M, K, seed=M)
    w = rnd(N, K, scale=0.05, seed=N + K)
    y = native.gemm_nt(x, w)
    ref = x.float() @ w.float().t()
    _check_bf16(y, ref)
    assert torch.equal(y, native.gemm_nt(x, w))


@pytest.mark.parametrize("M,N,K", [(6144, 1152, 896), (257, 1152, 896)])
def test_gemm_bias(M, N, K):
    x = rnd(M, K, seed=1)
    w = rnd(N, K, scale=0.05, seed=2)
    b = rnd(N, seed=3)
    y = native.gemm_nt(x, w, bias=b)
    ref = x.float() @ w.float().t() + b.float()
    _check_bf16(y, ref)


@pytest.mark.parametrize("M,I,K", [(6144, 4864, 896), (300, 4864, 896), (512, 64, 128)])
def test_gemm_swiglu(M, I, K):
    x = rnd(M, K, seed=5)
    w = rnd(2 * I, K, scale=0.05, seed=6)
    gu = torch.empty(M, 2 * I, dtype=BF, device=DEV)
    a = native.gemm_nt(x, w, swiglu=True, out_gu=gu)
    ref = x.float() @ w.float().t()
    _check_bf16(gu, ref)
    want = torch.empty(M, I, dtype=BF, device=DEV)
    native.swiglu_fwd(gu, want)  # the epilogue's math on the pre-activation it wrote
    assert torch.equal(a, want)
    a2 = native.gemm_nt(x, w, swiglu=True)  # no gu written: the same a
    assert torch.equal(a, a2)


@pytest.mark.parametrize("M,N,K", [(6144, 1152, 896), (4096, 896, 4864), (777, 9728, 896)])
def test_gemm_repeat_identical(M, N, K, tile):
    """race screen for the LDS-DMA / barrier schedule (cdna_hip_programming.md §5: an early read passes a single
    reference check whenever the copy happens to land first): 16 back-to-back launches, every result identical
    and within one rounding of the reference"""
    x = rnd(M, K, seed=11)
    w = rnd(N, K, scale=0.05, seed=12)
    y0 = native.gemm_nt(x, w)
    _check_bf16(y0, x.float() @ w.float().t())
    outs = [native.gemm_nt(x, w) for _ in range(16)]
    for y in outs:
        assert torch.equal(y, y0)
