"""drl_gemm (csrc/gemm_sk.hip): the forward / dgrad / wgrad GEMMs of nn.Linear (what F.linear and its autograd
backward compute under the reference's autocast, dp_actor.py:110) against a torch fp32 reference of the same op
on the same bf16 operands: every operand layout, the bf16 (plain / bias / SwiGLU) and fp32 (store / accumulate)
epilogues, ragged M / N / K, the stream-K split (few tiles, long K) and the whole-tile + stream-K mix, and the race
screen (repeated launches bit-identical, the split tiles summed in a fixed order)."""

import pytest
import torch

pytestmark = pytest.mark.gpu

from dots.rl_amd import native  # noqa: E402

K_, T_ = native.LAYOUT_K, native.LAYOUT_T


def _op(shape, layout, g, scale=1.0):
    """A bf16 operand holding the logical (rows, K) matrix in the given storage layout (+ a ragged row stride)."""
    r, k = shape
    if layout == K_:
        buf = torch.randn(r, k + 8, generator=g, device="cuda") * scale
        return buf.to(torch.bfloat16)[:, :k], lambda t: t.float()
    buf = torch.randn(k, (r + 15) // 8 * 8, generator=g, device="cuda") * scale  # ld % 8 == 0, > r
    return buf.to(torch.bfloat16)[:, :r], lambda t: t.float().t()


@pytest.fixture(autouse=True)
def _default_tuning():
    native.lib().drl_gemm_set_sk_tuning(0, 0, 0, 0)
    yield
    native.lib().drl_gemm_set_sk_tuning(0, 0, 0, 0)


@pytest.mark.parametrize("al,bl", [(K_, K_), (K_, T_), (T_, K_), (T_, T_)])
@pytest.mark.parametrize("M,N,K", [(300, 520, 256), (1024, 896, 1152), (96, 200, 4864), (2304, 2304, 384),
                                   (130, 700, 192), (777, 896, 896), (520, 1152, 64)])
def test_layouts_bf16_and_f32(al, bl, M, N, K):
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N + K + 3 * al + bl)
    a, fa = _op((M, K), al, g)
    b, fb = _op((N, K), bl, g)
    ref = fa(a).double() @ fb(b).double().t()
    tol = 4e-6 * K ** 0.5 * 1.0
    out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    native.gemm(a, al, b, bl, M, N, K, out)
    torch.testing.assert_close(out.double(), ref.to(torch.bfloat16).double(), rtol=8e-3, atol=tol)
    out32 = torch.full((M, N), 0.5, device="cuda")
    native.gemm(a, al, b, bl, M, N, K, out32, beta=True)
    torch.testing.assert_close(out32.double(), ref + 0.5, rtol=1e-6, atol=tol)
    native.gemm(a, al, b, bl, M, N, K, out32, beta=False)
    torch.testing.assert_close(out32.double(), ref, rtol=1e-6, atol=tol)


@pytest.mark.parametrize("al,bl,M,N,K,out", [(K_, K_, 65836, 896, 896, "bias"), (K_, T_, 82144, 896, 1152, "bf16"),
                                             (T_, T_, 16640, 1024, 520, "f32"), (K_, K_, 164288, 896, 4864, "bf16")])
def test_last_round_split_k(al, bl, M, N, K, out):
    """Whole-tile grids whose last round holds few tiles (n_tiles % 256 <= 64: the N = 896 outputs at the passes' token
    counts) split those tiles' K over the CUs (uniform split-K after the whole tiles, csrc/gemm_sk.hip tail mode):
    every epilogue kind against the fp64 product, and deterministic (split order fixed)."""
    g = torch.Generator(device="cuda").manual_seed(M + K)
    a, fa = _op((M, K), al, g, 0.5)
    b, fb = _op((N, K), bl, g, 0.5)
    tol = 4e-6 * K ** 0.5
    # the first rows and the last 1536 (the split tail tiles are the last ones): the fp64 product of those rows only
    rows = torch.cat([torch.arange(0, 512, device="cuda"), torch.arange(M - 1536, M, device="cuda")])
    ref = fa(a)[rows].double() @ fb(b).double().t()
    if out == "f32":
        c = torch.full((M, N), 0.25, device="cuda")
        native.gemm(a, al, b, bl, M, N, K, c, beta=True)
        torch.testing.assert_close(c[rows].double(), ref + 0.25, rtol=1e-6, atol=tol)
        c2 = torch.full((M, N), 0.25, device="cuda")
        native.gemm(a, al, b, bl, M, N, K, c2, beta=True)
        assert torch.equal(c, c2)
        return
    bias = torch.randn(N, generator=g, device="cuda").to(torch.bfloat16) if out == "bias" else None
    if bias is not None:
        ref = ref + bias.double()
    c = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    native.gemm(a, al, b, bl, M, N, K, c, bias=bias)
    torch.testing.assert_close(c[rows].double(), ref.to(torch.bfloat16).double(), rtol=8e-3, atol=tol)
    c2 = torch.empty_like(c)
    native.gemm(a, al, b, bl, M, N, K, c2, bias=bias)
    assert torch.equal(c, c2)


@pytest.mark.parametrize("K", [64, 200, 6144, 6150])
def test_wgrad_any_k(K):
    """Both operands layout T (the weight gradient over the token dimension): any token count, k tail zero."""
    g = torch.Generator(device="cuda").manual_seed(K)
    dy = torch.randn(K, 1152, generator=g, device="cuda").to(torch.bfloat16)
    x = torch.randn(K, 896, generator=g, device="cuda").to(torch.bfloat16)
    gw = torch.randn(1152, 896, generator=g, device="cuda")
    want = gw.double() + dy.double().t() @ x.double()
    native.linear_wgrad(gw, dy, x)
    torch.testing.assert_close(gw.double(), want, rtol=1e-6, atol=4e-6 * K ** 0.5)


def test_dgrad_reads_weight_in_place():
    g = torch.Generator(device="cuda").manual_seed(5)
    dy = torch.randn(6144, 9728, generator=g, device="cuda").to(torch.bfloat16)
    w = (torch.randn(9728, 896, generator=g, device="cuda") * 0.05).to(torch.bfloat16)
    dx = native.linear_dgrad(dy, w)
    ref = dy.float() @ w.float()
    torch.testing.assert_close(dx.float(), ref.to(torch.bfloat16).float(), rtol=8e-3, atol=1e-3)


@pytest.mark.parametrize("K", [72, 840, 1000])
def test_linear_reduction_not_multiple_of_64(K):
    """A model width that is not a multiple of 64 (the K tail): forward (with bias), input gradient and the SwiGLU-
    backward input gradient stay on drl_gemm through zero-padded operand copies (native._pad_to_64), no library
    fallback (qwen2.linear / dgrad)."""
    from dots.rl_amd import qwen2

    g = torch.Generator(device="cuda").manual_seed(K)
    x = torch.randn(300, K, generator=g, device="cuda").to(torch.bfloat16)
    w = (torch.randn(520, K, generator=g, device="cuda") * 0.05).to(torch.bfloat16)
    bias = torch.randn(520, generator=g, device="cuda").to(torch.bfloat16)
    y = qwen2.linear(x, w, bias=bias)
    ref = (x.double() @ w.double().t() + bias.double()).to(torch.bfloat16)
    torch.testing.assert_close(y.float(), ref.float(), rtol=8e-3, atol=1e-3)
    dy = torch.randn(300, K, generator=g, device="cuda").to(torch.bfloat16)
    wt = (torch.randn(K, 520, generator=g, device="cuda") * 0.05).to(torch.bfloat16)
    dx = qwen2.dgrad(dy, wt)
    torch.testing.assert_close(dx.float(), (dy.double() @ wt.double()).to(torch.bfloat16).float(), rtol=8e-3,
                               atol=1e-3)
    gu = torch.randn(300, 2 * 512, generator=g, device="cuda").to(torch.bfloat16)
    wd = (torch.randn(K, 512, generator=g, device="cuda") * 0.05).to(torch.bfloat16)
    dgu = native.linear_dgrad_swiglu_bwd(dy, wd, gu)
    da = native.linear_dgrad(dy, wd)
    want = torch.empty_like(gu)
    native.swiglu_bwd(gu, da, want)
    assert torch.equal(dgu, want)


def test_bf16_path_has_no_torch_fallback():
    from dots.rl_amd import qwen2

    with pytest.raises(NotImplementedError):
        qwen2.linear(torch.randn(4, 64, dtype=torch.float16, device="cuda"),
                     torch.randn(8, 64, dtype=torch.float16, device="cuda"))


@pytest.mark.parametrize("M", [256, 777, 6144])
def test_forward_epilogues(M):
    g = torch.Generator(device="cuda").manual_seed(M)
    x = torch.randn(M, 896, generator=g, device="cuda").to(torch.bfloat16)
    w = (torch.randn(1152, 896, generator=g, device="cuda") * 0.05).to(torch.bfloat16)
    bias = torch.randn(1152, generator=g, device="cuda").to(torch.bfloat16)
    y = native.linear_fwd(x, w, bias=bias)
    ref = (x.float() @ w.float().t() + bias.float()).to(torch.bfloat16)
    torch.testing.assert_close(y.float(), ref.float(), rtol=8e-3, atol=1e-3)
    wgu = (torch.randn(2 * 4864, 896, generator=g, device="cuda") * 0.05).to(torch.bfloat16)
    gu = torch.empty(M, 2 * 4864, dtype=torch.bfloat16, device="cuda")
    a = native.linear_fwd(x, wgu, swiglu=True, out_gu=gu)
    s = (x.float() @ wgu.float().t()).to(torch.bfloat16)
    torch.testing.assert_close(gu.float(), s.float(), rtol=8e-3, atol=1e-3)
    gg, uu = s[:, :4864].float(), s[:, 4864:].float()
    want = (torch.nn.functional.silu(gg).to(torch.bfloat16).float() * uu).to(torch.bfloat16)
    # the epilogue applies silu to ITS bf16 gate sum: compare against the reference built from the kernel's gu
    g2, u2 = gu[:, :4864].float(), gu[:, 4864:].float()
    want2 = (torch.nn.functional.silu(g2).to(torch.bfloat16).float() * u2).to(torch.bfloat16)
    torch.testing.assert_close(a.float(), want2.float(), rtol=1e-2, atol=1e-3)
    assert (a.float() - want.float()).abs().max() < 0.05 * want.float().abs().max()


@pytest.mark.parametrize("mode", [(0, 0, 0), (1, 0, 0), (2, 0, 0), (3, 0, 0), (3, 0, 5), (3, 0, 32), (1, 37, 0),
                                  (1, 7, 0)])
@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("K", [4864, 4800])
def test_decompositions_agree(mode, out_dtype, K):
    """Automatic, stream-K, whole tiles, uniform split-K (automatic / 5 / 32 splits), odd grids: the same GEMM
    within fp32 summation-order differences. K = 4800: an odd k-tile count (the last pair's empty second tile is
    skipped by whichever segment holds it)."""
    dp_mode, grid, param = mode
    g = torch.Generator(device="cuda").manual_seed(11)
    a = torch.randn(1000, K, generator=g, device="cuda").to(torch.bfloat16)
    b = torch.randn(896, K, generator=g, device="cuda").to(torch.bfloat16)
    bias = torch.randn(896, generator=g, device="cuda").to(torch.bfloat16) if out_dtype == torch.bfloat16 else None
    ref = a.double() @ b.double().t() + (bias.double() if bias is not None else 0)
    native.lib().drl_gemm_set_sk_tuning(grid, 0, dp_mode, param)
    out = torch.empty(1000, 896, device="cuda", dtype=out_dtype)
    native.gemm(a, K_, b, K_, 1000, 896, K, out, bias=bias)
    if out_dtype == torch.float32:
        torch.testing.assert_close(out.double(), ref, rtol=1e-6, atol=4e-6 * K ** 0.5)
    else:
        torch.testing.assert_close(out.double(), ref.to(torch.bfloat16).double(), rtol=8e-3, atol=4e-6 * K ** 0.5)


@pytest.mark.parametrize("al,bl,M,N,K", [(K_, K_, 6144, 896, 4864), (K_, T_, 2048, 896, 37888),
                                         (T_, T_, 896, 896, 6144), (K_, K_, 6144, 9728, 896),
                                         (K_, K_, 16640, 1024, 4096)])
@pytest.mark.parametrize("mode", [(0, 0), (1, 0), (3, 4)])
def test_race_screen(al, bl, M, N, K, mode):
    """16 launches bit-identical (split tiles are reduced in k order, whatever the arrival order). 16640 x 1024 x 4096
    under the automatic plan is the tail split-K form (260 tiles = 256 + 4 over 256 CUs: a grid above the CU count),
    whose timeout word sits at the fixed index flags + CU count (read back below)."""
    native.lib().drl_gemm_set_sk_tuning(0, 0, mode[0], mode[1])
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    a, _ = _op((M, K), al, g)
    b, _ = _op((N, K), bl, g)
    outs = []
    for _ in range(16):
        o = torch.empty(M, N, device="cuda")
        native.gemm(a, al, b, bl, M, N, K, o)
        outs.append(o)
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    ws = native._ws_gemm.get(outs[0].device)
    n = native.lib().drl_gemm_workspace_bytes()
    cus = (n - 256) // (256 * 256 * 4 + 4)
    flags = ws[cus * 256 * 256 * 4:].view(torch.int32)[:cus + 1]
    assert int(flags.abs().sum()) == 0  # every flag consumed and reset, no residency timeout recorded
    assert native.gemm_timeout_word(outs[0].device) == 0


def test_operand_over_2gb_rebases_per_tile():
    """The prefill's down_proj input (512 x 512 rows x 4864) is 2.5 GB, past one buffer range: drl_gemm runs one
    launch whose A descriptor is rebased per tile row; spot rows (first / last tiles, round-4 block edges) against the
    fp32 reference."""
    M, N, K = 262144, 896, 4864
    g = torch.Generator(device="cuda").manual_seed(3)
    a = torch.empty(M, K, dtype=torch.bfloat16, device="cuda")
    a.copy_(torch.randn(1, K, generator=g, device="cuda").expand(M, K))
    a[:, :64] = torch.randn(M, 64, generator=g, device="cuda").to(torch.bfloat16)  # every row different
    b = (torch.randn(N, K, generator=g, device="cuda") * 0.05).to(torch.bfloat16)
    out = native.linear_fwd(a, b)
    rows = torch.tensor([0, 1, 255, 256, 200000, 220000, 220671, 220672, M - 1], device="cuda")
    ref = a[rows].float() @ b.float().t()
    torch.testing.assert_close(out[rows].float(), ref.to(torch.bfloat16).float(), rtol=8e-3, atol=2e-3)
    del a, out


@pytest.mark.parametrize("M", [7000, 7168])
def test_lm_head_dgrad_operand_over_2gb(M):
    """The lm_head input gradient: d_logits (M x 151936 bf16, > 2 GB) as the layout-K A operand of dx = dy W with
    W (151936, 896) layout T — one launch, A rebased per tile; the last tile's rows past M read as zeros (M = 7000).
    Spot rows against fp32 torch."""
    K, N = 151936, 896
    g = torch.Generator(device="cuda").manual_seed(M)
    dy = torch.randn(M, K, generator=g, device="cuda").to(torch.bfloat16)
    w = (torch.randn(K, N, generator=g, device="cuda") * 0.05).to(torch.bfloat16)
    dx = native.linear_dgrad(dy, w)
    rows = torch.tensor([0, 255, 256, 3333, 6655, 6656, M - 2, M - 1], device="cuda")
    ref = dy[rows].float() @ w.float()
    torch.testing.assert_close(dx[rows].float(), ref.to(torch.bfloat16).float(), rtol=1e-2, atol=2e-2)
    del dy, dx


def test_wgrad_operand_over_2gb_splits_k():
    """The fused-micro-batch lm_head weight gradient: d_logits (8448 tokens x 131072 vocab, bf16, 2.2 GB) read as a
    layout-T operand past one buffer range: drl_gemm accumulates K blocks into the fp32 gradient. Spot rows of the
    result against fp32 torch, starting from a non-zero gradient (beta = 1)."""
    T_, V, H = 8448, 131072, 64
    g = torch.Generator(device="cuda").manual_seed(5)
    dy = torch.randn(T_, V, generator=g, device="cuda").to(torch.bfloat16)
    x = torch.randn(T_, H, generator=g, device="cuda").to(torch.bfloat16)
    gw = torch.ones(V, H, device="cuda")
    native.linear_wgrad(gw, dy, x)
    rows = torch.tensor([0, 1, 77, 65535, 65536, V - 1], device="cuda")
    ref = 1.0 + dy[:, rows].float().t() @ x.float()
    torch.testing.assert_close(gw[rows], ref, rtol=1e-4, atol=1e-3)
    del dy, gw


@pytest.mark.parametrize("M,N_out,N_in", [(6144, 1152, 896), (6144, 9728, 896), (6144, 896, 4864), (777, 896, 896),
                                         (82144, 896, 896)])
def test_concurrent_dgrad_wgrad_matches_serial(M, N_out, N_in, monkeypatch):
    """qwen2.dgrad_wgrad: the weight gradient on the side stream (workspace slot 1) while the input gradient runs on
    the current stream gives bit-identical results to the serial pair, repeated back to back (slots reused)."""
    from dots.rl_amd import qwen2

    monkeypatch.setattr(qwen2, "CONCURRENT_WGRAD", True)
    # every shape through the side stream, including the split-K weight gradients qwen2 now runs in sequence
    monkeypatch.setattr(qwen2, "_concurrent_pair", lambda gw: True)

    g = torch.Generator(device="cuda").manual_seed(M + N_out)
    dy = torch.randn(M, N_out, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(N_out, N_in, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
    x = torch.randn(M, N_in, device="cuda", generator=g).to(torch.bfloat16)
    gw0 = torch.randn(N_out, N_in, device="cuda", generator=g)
    gw_s, gw_c = gw0.clone(), gw0.clone()
    for _ in range(3):
        dx_s = native.linear_dgrad(dy, w)
        native.linear_wgrad(gw_s, dy, x)
        dx_c = qwen2.dgrad_wgrad(dy, w, gw_c, x)
    torch.cuda.synchronize()
    assert torch.equal(dx_s, dx_c)
    assert torch.equal(gw_s, gw_c)


@pytest.mark.parametrize("M", [6144, 777, 24576])
def test_dgrad_swiglu_bwd_epilogue_matches_unfused(M):
    """The down_proj dgrad with the SwiGLU backward in its epilogue (dgu straight from the accumulators and the saved
    gu) equals dgrad -> bf16 d a -> swiglu_bwd bit for bit (K = 896: both run whole tiles, one summation order)."""
    I, H = 4864, 896
    g = torch.Generator(device="cuda").manual_seed(M)
    dm = torch.randn(M, H, generator=g, device="cuda").to(torch.bfloat16)
    w = (torch.randn(H, I, generator=g, device="cuda") * 0.05).to(torch.bfloat16)
    gu = (torch.randn(M, 2 * I, generator=g, device="cuda") * 2).to(torch.bfloat16)
    da = native.linear_dgrad(dm, w)
    want = torch.empty_like(gu)
    native.swiglu_bwd(gu, da, want)
    got = native.linear_dgrad_swiglu_bwd(dm, w, gu)
    assert torch.equal(got, want)
    # strided / ragged: a view of wider rows, I not a multiple of the tile
    I2 = 4864 - 96
    w2 = w[:, :I2].contiguous()
    gu2 = torch.cat([gu[:, :I2], gu[:, I:I + I2]], 1)
    da2 = native.linear_dgrad(dm, w2)
    want2 = torch.empty_like(gu2)
    native.swiglu_bwd(gu2, da2, want2)
    assert torch.equal(native.linear_dgrad_swiglu_bwd(dm, w2, gu2), want2)


@pytest.mark.parametrize("M", [14000])
def test_swiglu_forward_stream_k_matches_whole_tiles(M):
    """The gate_up + SwiGLU forward over >= 8 rounds of tiles runs persistent whole-tile rounds + a stream-K tail
    (automatic); against one workgroup per tile (forced whole tiles): gu within one bf16 rounding of the fp32 sums
    (only the tail's split tiles sum in another order), the SwiGLU output built from the kernel's own gu, and 8
    launches bit-identical (k-order combine)."""
    g = torch.Generator(device="cuda").manual_seed(M)
    x = torch.randn(M, 896, generator=g, device="cuda").to(torch.bfloat16)
    wgu = (torch.randn(2 * 4864, 896, generator=g, device="cuda") * 0.05).to(torch.bfloat16)
    gu = torch.empty(M, 2 * 4864, dtype=torch.bfloat16, device="cuda")
    a = native.linear_fwd(x, wgu, swiglu=True, out_gu=gu)
    for _ in range(8):
        gu2 = torch.empty_like(gu)
        assert torch.equal(native.linear_fwd(x, wgu, swiglu=True, out_gu=gu2), a)
        assert torch.equal(gu2, gu)
    native.lib().drl_gemm_set_sk_tuning(0, 0, 2, 0)
    try:
        guw = torch.empty_like(gu)
        aw = native.linear_fwd(x, wgu, swiglu=True, out_gu=guw)
    finally:
        native.lib().drl_gemm_set_sk_tuning(0, 0, 0, 0)
    s = (x.float() @ wgu.float().t())
    torch.testing.assert_close(gu.float(), s, rtol=8e-3, atol=1e-3)
    assert (gu.float() - guw.float()).abs().max() <= 8e-3 * s.abs().max()
    g2, u2 = gu[:, :4864].float(), gu[:, 4864:].float()
    want = (torch.nn.functional.silu(g2).to(torch.bfloat16).float() * u2).to(torch.bfloat16)
    torch.testing.assert_close(a.float(), want.float(), rtol=1e-2, atol=1e-3)
    same = gu == guw
    assert same.float().mean() > 0.9  # whole-tile rounds give the same bits; only the tail's split tiles may differ
    assert torch.equal(a[same[:, :4864] & same[:, 4864:]], aw[same[:, :4864] & same[:, 4864:]])


@pytest.mark.parametrize("T", [82144])
def test_down_wgrad_automatic_split_k(T):
    """down_proj's weight gradient over the update pass's tokens (76 tiles x 642 k-pairs) takes 3 uniform split-K
    slices automatically: against fp32 torch (accumulated onto a non-zero gradient), and reproducible bit for bit."""
    g = torch.Generator(device="cuda").manual_seed(T)
    dy = torch.randn(T, 896, generator=g, device="cuda").to(torch.bfloat16)
    x = torch.randn(T, 4864, generator=g, device="cuda").to(torch.bfloat16)
    gw = torch.full((896, 4864), 0.5, device="cuda")
    native.linear_wgrad(gw, dy, x)
    ref = 0.5 + dy.double().t() @ x.double()  # fp64: the fp32 sums' summation-order error alone, ~1e-5 sqrt(T)
    torch.testing.assert_close(gw.double(), ref, rtol=1e-6, atol=1e-5 * T ** 0.5)
    gw2 = torch.full((896, 4864), 0.5, device="cuda")
    native.linear_wgrad(gw2, dy, x)
    assert torch.equal(gw, gw2)


def test_layout_t_operand_over_2gb_walks_k_in_one_launch():
    """The lm_head weight gradient's d_logits^T (T x V bf16 past one 2 GB buffer range, layout T) as ONE launch whose
    tiles walk K in blocks with the A descriptor rebased per block (round 6; round 5 launched one GEMM per K block, each
    a read-modify-write of the fp32 output): against the K-block host loop (drl_gemm_set_debug bit 16, fp32 sums
    rounded per block) within fp32 rounding, and spot rows against fp64; beta accumulates."""
    T, V, H = 8192, 151936, 896
    g = torch.Generator(device="cuda").manual_seed(5)
    dy = torch.empty(T, V, dtype=torch.bfloat16, device="cuda")
    for r0 in range(0, T, 1024):  # fill in slices (bounded temporaries)
        dy[r0:r0 + 1024] = (torch.randn(1024, V, generator=g, device="cuda") * 0.1).to(torch.bfloat16)
    x = torch.randn(T, H, generator=g, device="cuda").to(torch.bfloat16)
    base = torch.randn(V, H, generator=g, device="cuda")
    gw = base.clone()
    native.linear_wgrad(gw, dy, x)  # one launch, K blocks inside
    gw2 = base.clone()
    native.lib().drl_gemm_set_debug(16)
    try:
        native.linear_wgrad(gw2, dy, x)  # the host loop of K-block launches
    finally:
        native.lib().drl_gemm_set_debug(0)
    torch.testing.assert_close(gw, gw2, rtol=1e-5, atol=1e-4)
    rows = torch.tensor([0, 1, 255, 256, 70000, V - 1], device="cuda")
    ref = base[rows].double() + dy[:, rows].double().t() @ x.double()
    torch.testing.assert_close(gw[rows].double(), ref, rtol=1e-5, atol=2e-4)
    gw3 = base.clone()
    native.linear_wgrad(gw3, dy, x)
    assert torch.equal(gw, gw3)  # deterministic
    del dy


@pytest.mark.parametrize("al,bl", [(K_, K_), (K_, T_), (T_, K_), (T_, T_)])
@pytest.mark.parametrize("M,N,K", [(777, 896, 896), (520, 1152, 320), (300, 520, 1280), (2304, 384, 640),
                                   (16640, 896, 2048)])
def test_half_width_last_tile_column_bit_identical(al, bl, M, N, K):
    """The last tile column of N % 256 in (0, 128] (the N = 896 / 1152 outputs) runs half-width tiles: B's 128 columns
    in one LDS half, the other quadrant's MFMAs skipped (csrc/gemm_sk.hip, setup_tile hn). Same k order per output, so
    the bf16 (plain / bias) and fp32 (store / accumulate) results equal the full-width tiles' bit for bit (debug bit
    32 forces the full-width path)."""
    g = torch.Generator(device="cuda").manual_seed(M + 3 * N + K + al + 5 * bl)
    a, fa = _op((M, K), al, g)
    b, fb = _op((N, K), bl, g)
    bias = torch.randn(N, generator=g, device="cuda").to(torch.bfloat16) if al == K_ and bl == K_ else None
    c0 = torch.randn(M, N, generator=g, device="cuda")
    res = []
    try:
        for dbg in (0, 32):
            native.lib().drl_gemm_set_debug(dbg)
            out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
            native.gemm(a, al, b, bl, M, N, K, out, bias=bias)
            out32 = c0.clone()
            native.gemm(a, al, b, bl, M, N, K, out32, beta=True)
            res.append((out, out32))
    finally:
        native.lib().drl_gemm_set_debug(0)
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1])
    ref = fa(a).double() @ fb(b).double().t() + (bias.double() if bias is not None else 0.0)
    torch.testing.assert_close(res[0][0].double(), ref.to(torch.bfloat16).double(), rtol=8e-3,
                               atol=4e-6 * K ** 0.5 + 1e-2 * (bias is not None))
