"""The fused attention backward at the update pass's shapes (B x 2 KV heads x 7 query heads, T = 768, head_dim 64;
B = 256 with 7 of 8 rows skipping query tiles below 512 = prefix sharing), per dQ variant
(drl_flash_attn_bwd_set_variant: 0 one query tile per workgroup, 1 two tiles with K / V in registers, 2 two tiles
re-reading K / V): mean of 5 x 10 calls. python tools/probes/flash_dq_ab.py"""
import json
import sys

import torch

sys.path.insert(0, ".")
from dots.rl_amd import native  # noqa: E402

dev, bf = "cuda", torch.bfloat16
lib = native.lib()
for B, qs in ((32, None), (256, 512)):
    Hkv, G, D, T = 2, 7, 64, 768
    g = torch.Generator(device=dev).manual_seed(B)
    q = torch.randn(B, Hkv, G, T, D, device=dev, generator=g).to(bf)
    k = torch.randn(B, Hkv, T, D, device=dev, generator=g).to(bf)
    v = torch.randn(B, Hkv, T, D, device=dev, generator=g).to(bf)
    kt = k.transpose(-1, -2).contiguous()
    vt = v.transpose(-1, -2).contiguous()
    valid = torch.ones(B, T, dtype=torch.uint8, device=dev)
    valid[1::3, :17] = 0
    q_start = None
    if qs is not None:
        q_start = torch.zeros(B, dtype=torch.int32, device=dev)
        q_start[torch.arange(B, device=dev) % 8 != 0] = qs
    o = torch.empty(B, T, Hkv * G * D, device=dev, dtype=bf)
    lse = torch.empty(B, Hkv, G, T, device=dev)
    native.flash_attn_fwd(q, k, vt, valid, o, lse=lse, q_start=q_start)
    dout = torch.randn(B, T, Hkv * G * D, device=dev, generator=g).to(bf)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    row = {"B": B, "q_start": qs}
    for var in (0, 1, 2):
        lib.drl_flash_attn_bwd_set_variant(var)
        fn = lambda: native.flash_attn_bwd(q, k, kt, v, o, dout, lse, valid, dq, dk, dv, q_start=q_start)  # noqa: E731
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 100)
        row[f"bwd_var{var}_us"] = round(sorted(ts)[2], 1)
    lib.drl_flash_attn_bwd_set_variant(0)
    print(json.dumps(row), flush=True)
