"""The decode lm_head at the N = 8 rank's 64 rows (and 32 / 1): the persistent decode kernel vs drl_gemm on the same
operands, graph-replayed (8 weight copies rotated: cold, > MALL). python tools/probes/lm_head64.py"""
import json
import sys

import torch

sys.path.insert(0, ".")
from dots.rl_amd import native  # noqa: E402

DEV, BF = "cuda", torch.bfloat16
V, K = 151936, 896
ws = [(torch.randn(V, K, device=DEV) * 0.05).to(BF) for _ in range(4)]
wps = [native.decode_pack_weight(w) for w in ws]
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def gt(fn, calls=16):
    fn(0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        g.capture_begin()
        for i in range(calls):
            fn(i)
        g.capture_end()
    torch.cuda.synchronize()
    for _ in range(2):
        a.record()
        g.replay()
        b.record()
        b.synchronize()
    return round(a.elapsed_time(b) * 1e3 / calls, 2)


for M in (64, 32, 1):
    mbt = native.decode_lm_head_plan(M, V, K)
    h = torch.randn(M, K, device=DEV).to(BF)
    hp = native.pack_activations(h, mbt)
    out = torch.empty(M, V, dtype=BF, device=DEV)
    row = {"rows": M}
    for ci in range(6):
        native.lib().drl_decode_lm_head_set_config(ci)
        t = gt(lambda i: native.decode_lm_head(hp, mbt, wps[i % 4], M, V, K, out))
        row[f"decode_cfg{ci}_us"] = t
        row[f"decode_cfg{ci}_TBps"] = round(V * K * 2 / t / 1e6, 2)
    native.lib().drl_decode_lm_head_set_config(-1)
    row["decode_auto_us"] = gt(lambda i: native.decode_lm_head(hp, mbt, wps[i % 4], M, V, K, out))
    t_gemm = gt(lambda i: native.linear_fwd(h, ws[i % 4], out=out))
    row.update(drl_gemm_us=t_gemm, gemm_TBps=round(V * K * 2 / t_gemm / 1e6, 2))
    print(json.dumps(row), flush=True)
