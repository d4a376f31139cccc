"""hipBLASLt (replayed TunableOp choices) on the update micro-batch GEMMs in each call form: forward x W^T,
dgrad dy W (NN) vs dy (W^T)^T with a pre-transposed weight (TN), wgrad dy^T x (fp32 accumulate) vs
dy^T-contiguous @ (x^T-contiguous)^T (TN) with the transposes timed separately. us per call."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import json

import torch

from dots.rl_amd.workers import _enable_gemm_tuning

_enable_gemm_tuning("auto")


def t_it(fn, n=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / n * 1e3


bf = torch.bfloat16
for name, N, K in (("qkv", 1152, 896), ("o", 896, 896), ("gate_up", 9728, 896), ("down", 896, 4864)):
    M = 6144
    x = torch.randn(M, K, device="cuda", dtype=bf)
    w = torch.randn(N, K, device="cuda", dtype=bf) * 0.05
    dy = torch.randn(M, N, device="cuda", dtype=bf)
    gw = torch.zeros(N, K, device="cuda")
    wt = w.t().contiguous()
    fl = 2.0 * M * N * K
    r = dict(layer=name, M=M, N=N, K=K)
    r["fwd"] = t_it(lambda: x @ w.t())
    r["dgrad_nn"] = t_it(lambda: dy @ w)
    r["dgrad_tn_wT"] = t_it(lambda: dy @ wt.t())
    r["wgrad_cur"] = t_it(lambda: torch.addmm(gw, dy.t(), x, out_dtype=torch.float32, out=gw))
    dyt = dy.t().contiguous()
    xt = x.t().contiguous()
    r["wgrad_tn"] = t_it(lambda: torch.addmm(gw, dyt, xt.t(), out_dtype=torch.float32, out=gw))
    r["wgrad_tn_bf16out"] = t_it(lambda: dyt @ xt.t())
    r["transpose_dy"] = t_it(lambda: dy.t().contiguous())
    r["transpose_x"] = t_it(lambda: x.t().contiguous())
    r["TF"] = {k: round(fl / v / 1e6) for k, v in r.items() if k in ("fwd", "dgrad_nn", "dgrad_tn_wT", "wgrad_cur", "wgrad_tn", "wgrad_tn_bf16out")}
    print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
