"""Fused attention kernels alone, for counter passes (rocprofv3 --pmc): forward at the log-prob shape (B = 80) and
backward at the update shape (B = 32), T = 768, Qwen2.5-0.5B heads, 5 launches each.
  python tools/probes/flash_probe.py [fwd|bwd|both]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dots.rl_amd import native  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "both"
dev, bf = "cuda", torch.bfloat16
Hkv, G, D, T = 2, 7, 64, 768
for B, kind in ((80, "fwd"), (32, "bwd")):
    if which not in (kind, "both"):
        continue
    q = torch.randn(B, Hkv, G, T, D, device=dev, dtype=bf)
    k = torch.randn(B, Hkv, T, D, device=dev, dtype=bf)
    v = torch.randn(B, Hkv, T, D, device=dev, dtype=bf)
    kt, vt = k.transpose(-1, -2).contiguous(), v.transpose(-1, -2).contiguous()
    valid = torch.ones(B, T, dtype=torch.uint8, device=dev)
    o = torch.empty(B, T, Hkv * G * D, device=dev, dtype=bf)
    lse = torch.empty(B, Hkv, G, T, device=dev)
    native.flash_attn_fwd(q, k, vt, valid, o, lse=lse)
    dout = torch.randn_like(o)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    for _ in range(5):
        if kind == "fwd":
            native.flash_attn_fwd(q, k, vt, valid, o, lse=lse)
        else:
            native.flash_attn_bwd(q, k, kt, v, o, dout, lse, valid, dq, dk, dv)
    torch.cuda.synchronize()
print("ok")
