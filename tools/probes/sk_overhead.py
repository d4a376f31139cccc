"""Per-tile fixed cost of drl_gemm: the same tile grid at K = 896 / 1792 / 3584 (T(K) = fixed + K * rate), plain /
SwiGLU / bias epilogues, at the update pass's gate_up shape (24576 x 9728) and the N = 896 forward (24576 x 896)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from gemm_sk_bench import bench  # noqa: E402
from dots.rl_amd import native  # noqa: E402

bf = torch.bfloat16
for M, N in [tuple(int(v) for v in a.split('x')) for a in sys.argv[1:]] or ((24576, 9728), (24576, 896), (61440, 9728)):
    for K in (896, 1792):
        x = torch.randn(M, K, device="cuda", dtype=bf)
        w = torch.randn(N, K, device="cuda", dtype=bf) * 0.05
        b = torch.randn(N, device="cuda", dtype=bf)
        row = dict(M=M, N=N, K=K)
        row["plain_us"] = round(bench(lambda: native.linear_fwd(x, w)), 1)
        native.lib().drl_gemm_set_debug(1)
        row["no_epilogue_us"] = round(bench(lambda: native.linear_fwd(x, w)), 1)
        native.lib().drl_gemm_set_debug(4)
        row["barriers_only_us"] = round(bench(lambda: native.linear_fwd(x, w)), 1)
        native.lib().drl_gemm_set_debug(2)
        row["stage_no_store_us"] = round(bench(lambda: native.linear_fwd(x, w)), 1)
        native.lib().drl_gemm_set_debug(0)
        row["bias_us"] = round(bench(lambda: native.linear_fwd(x, w, bias=b)), 1)
        if N % 64 == 0 and N > 1000:
            row["swiglu_us"] = round(bench(lambda: native.linear_fwd(x, w, swiglu=True)), 1)
        tiles = ((M + 255) // 256) * ((N + 255) // 256)
        row["tiles"] = tiles
        print(json.dumps(row), flush=True)
