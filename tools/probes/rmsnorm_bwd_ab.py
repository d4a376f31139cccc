"""A/B of the RMSNorm backward (csrc/layers.hip rmsnorm_bwd_vec_kernel) between two builds of the library: output
hashes (dx, dx_bf16, dw on seeded inputs) and time per call at the update pass's row counts.

  DOTSRL_AMD_LIB=<lib.so> python tools/probes/rmsnorm_bwd_ab.py
"""
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dots.rl_amd import native  # noqa: E402

H = 896
for N in (82144, 164288, 16384 + 3):
    g = torch.Generator(device="cuda").manual_seed(N)
    x = torch.randn(N, H, device="cuda", generator=g)
    w = torch.randn(H, device="cuda", generator=g)
    rstd = torch.rsqrt(x.pow(2).mean(-1) + 1e-6)
    dy = torch.randn(N, H, device="cuda", generator=g).to(torch.bfloat16)
    dx_in = torch.randn(N, H, device="cuda", generator=g)
    dx = torch.empty_like(x)
    dxb = torch.empty(N, H, device="cuda", dtype=torch.bfloat16)
    dw = torch.zeros(H, device="cuda")
    native.rmsnorm_bwd(x, w, rstd, dy, dx, dw, dx_in=dx_in, dx_bf16=dxb)
    torch.cuda.synchronize()
    h = hashlib.sha1()
    for t in (dx, dxb, dw):
        h.update(t.view(torch.uint8).cpu().numpy().tobytes() if t.dtype != torch.bfloat16
                 else t.view(torch.int16).cpu().numpy().tobytes())
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        native.rmsnorm_bwd(x, w, rstd, dy, dx, dw, dx_in=dx_in, dx_bf16=dxb)
    a.record()
    for _ in range(20):
        native.rmsnorm_bwd(x, w, rstd, dy, dx, dw, dx_in=dx_in, dx_bf16=dxb)
    b.record()
    b.synchronize()
    us = a.elapsed_time(b) * 1e3 / 20
    byt = N * H * 16
    print(json.dumps({"lib": os.path.basename(os.environ.get("DOTSRL_AMD_LIB", "libdotsrl_amd.so")), "N": N,
                      "us": round(us, 1), "TBps": round(byt / us / 1e6, 2), "sha1": h.hexdigest()[:16]}), flush=True)
