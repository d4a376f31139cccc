"""A/B of the fused attention kernels between two builds of the library (DRL_LIB_PATH selects the build): forward
and backward at the update pass's shape (B sequences x 2 KV heads x 7 query heads, T = 768, head_dim 64, with and
without a q_start skip), outputs saved for a bitwise comparison and timed.

  DRL_LIB_PATH=<so> python tools/probes/flash_ab.py run <tag>   -> /tmp/flash_ab_<tag>.pt + one JSON line
  python tools/probes/flash_ab.py cmp <tag1> <tag2>             -> bitwise equality of every output"""

import json
import os
import sys

import torch

sys.path.insert(0, ".")

if sys.argv[1] == "cmp":
    a = torch.load(f"/tmp/flash_ab_{sys.argv[2]}.pt", weights_only=True)
    b = torch.load(f"/tmp/flash_ab_{sys.argv[3]}.pt", weights_only=True)
    print(json.dumps({k: bool(torch.equal(a[k], b[k])) for k in a}))
    sys.exit(0)

from dots.rl_amd import native  # noqa: E402

tag = sys.argv[2]
dev, bf = "cuda", torch.bfloat16
out = {}
res = {}
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
    if qs is not None:  # prefix sharing: 7 of every 8 rows skip their query tiles below qs
        q_start = torch.zeros(B, dtype=torch.int32, device=dev)
        q_start[torch.arange(B, device=dev) % 8 != 0] = qs
    o = torch.empty(B, T, Hkv * G * D, device=dev, dtype=bf)
    lse = torch.empty(B, Hkv, G, T, device=dev)
    native.flash_attn_fwd(q, k, vt, valid, o, lse=lse, q_start=q_start)
    dout = torch.randn(B, T, Hkv * G * D, device=dev, generator=g).to(bf)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    bwd = lambda: native.flash_attn_bwd(q, k, kt, v, o, dout, lse, valid, dq, dk, dv, q_start=q_start)  # noqa: E731
    fwd = lambda: native.flash_attn_fwd(q, k, vt, valid, o, lse=lse, q_start=q_start)  # noqa: E731
    for name, fn in (("fwd", fwd), ("bwd", bwd)):
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
            ts.append(e0.elapsed_time(e1) * 1e3 / 10)
        res[f"{name}_B{B}_us"] = round(sorted(ts)[2], 1)
    out.update({f"o{B}": o.clone(), f"lse{B}": lse.clone(), f"dq{B}": dq.clone(), f"dk{B}": dk.clone(),
                f"dv{B}": dv.clone()})
pass
torch.save(out, f"/tmp/flash_ab_{tag}.pt")
print(json.dumps(dict(tag=tag, lib=os.environ.get("DRL_LIB_PATH"), **res)), flush=True)
