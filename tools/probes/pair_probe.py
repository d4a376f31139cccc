"""The gate_up projection's input + weight gradient pair at the update pass's 82144 rows (dy (T, 9728), w (9728, 896),
x (T, 896), gw fp32 (9728, 896)): concurrent (qwen2.dgrad_wgrad, the product schedule) against the two in sequence
with the weight gradient as whole tiles (152 tiles over 256 CUs) or as uniform split-K with S slabs per tile.

  python tools/probes/pair_probe.py [T]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dots.rl_amd import native, qwen2  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 82144
bf = torch.bfloat16
shapes = {"gate_up": (9728, 896), "down": (896, 4864)}
lib = native.lib()


def timed(fn, reps=6):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


for name, (O, I) in shapes.items():
    g = torch.Generator(device="cuda").manual_seed(O)
    dy = torch.randn(T, O, device="cuda", dtype=bf, generator=g)
    w = (torch.randn(O, I, device="cuda", generator=g) * 0.05).to(bf)
    x = torch.randn(T, I, device="cuda", dtype=bf, generator=g)
    gw = torch.zeros(O, I, device="cuda")
    row = {"pair": name, "T": T}
    row["concurrent_us" if qwen2._concurrent_pair(gw) else "product_sequential_us"] = round(
        timed(lambda: qwen2.dgrad_wgrad(dy, w, gw, x)), 1)
    row["dgrad_us"] = round(timed(lambda: native.linear_dgrad(dy, w)), 1)
    row["wgrad_auto_us"] = round(timed(lambda: native.linear_wgrad(gw, dy, x)), 1)
    ref = torch.zeros_like(gw)
    native.linear_wgrad(ref, dy, x)
    for S in (2, 3, 4, 5, 6, 8):
        lib.drl_gemm_set_sk_tuning(0, 0, 3, S)
        try:
            row[f"wgrad_S{S}_us"] = round(timed(lambda: native.linear_wgrad(gw, dy, x)), 1)
            chk = torch.zeros_like(gw)
            native.linear_wgrad(chk, dy, x)
            row[f"wgrad_S{S}_relerr"] = float((chk - ref).abs().max() / ref.abs().max())
        finally:
            lib.drl_gemm_set_sk_tuning(0, 0, 0, 0)
    print(json.dumps(row), flush=True)
