"""Error pattern of drl_gemm_bf16_nt vs the fp32 product (debug aid)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from dots.rl_amd import native
BF = torch.bfloat16
for (M, N, K, tile) in [(6144, 896, 896, t) for t in (1, 2, 3, 4, 5)] + [(300, 200, 128, t) for t in (3, 4, 5)]:
    native.lib().drl_gemm_set_tile(tile)
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(M, K, device="cuda", generator=g).to(BF)
    w = (torch.randn(N, K, device="cuda", generator=g) * 0.05).to(BF)
    y = native.gemm_nt(x, w).float()
    ref = x.float() @ w.float().t()
    err = (y - ref).abs()
    bad = err > ref.abs() * 2 ** -7 * 1.01 + 1e-6
    print(M, N, K, tile, "max err", err.max().item(), "bad frac", bad.float().mean().item())
    if bad.any():
        idx = bad.nonzero()
        print("  bad rows mod 32:", torch.bincount(idx[:, 0] % 32, minlength=32).tolist())
        print("  bad cols mod 32:", torch.bincount(idx[:, 1] % 32, minlength=32).tolist())
        print("  bad rows //32 (first 16):", torch.bincount(idx[:, 0] // 32)[:16].tolist())
        i, j = idx[0].tolist()
        print("  e.g.", i, j, y[i, j].item(), ref[i, j].item())
native.lib().drl_gemm_set_tile(0)
