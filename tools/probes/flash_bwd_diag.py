"""Localise a fused-attention backward mismatch: per 32-key tile max error of dk / dv (and per 32-query tile of
dq) against fp32 autograd, at one shape. python tools/probes/flash_bwd_diag.py B Hkv G D T"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dots.rl_amd import native  # noqa: E402

B, Hkv, G, D, T = (int(x) for x in sys.argv[1:6])
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(T + G)
q = torch.randn(B, Hkv, G, T, D, device=dev, generator=g).to(torch.bfloat16)
k = torch.randn(B, Hkv, T, D, device=dev, generator=g).to(torch.bfloat16)
v = torch.randn(B, Hkv, T, D, device=dev, generator=g).to(torch.bfloat16)
dout = torch.randn(B, T, Hkv * G * D, device=dev, generator=g).to(torch.bfloat16)
valid = torch.zeros(B, (T + 3) // 4 * 4, dtype=torch.uint8, device=dev)
valid[:, :T] = 1
ld = (T + 7) // 8 * 8
kt = torch.zeros(B, Hkv, D, ld, device=dev, dtype=torch.bfloat16)
kt[..., :T] = k.transpose(-1, -2)
vt = torch.zeros_like(kt)
vt[..., :T] = v.transpose(-1, -2)
o = torch.empty(B, T, Hkv * G * D, device=dev, dtype=torch.bfloat16)
lse = torch.empty(B, Hkv, G, T, device=dev)
native.flash_attn_fwd(q, k, vt, valid, o, lse=lse)
dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
native.flash_attn_bwd(q, k, kt, v, o, dout, lse, valid, dq, dk, dv)
qf, kf, vf = (t.float().requires_grad_(True) for t in (q, k, v))
S = torch.einsum("bhgtd,bhkd->bhgtk", qf, kf) / math.sqrt(D)
j = torch.arange(T, device=dev)
allowed = (j <= j[:, None])[None, None, None]
P = torch.softmax(S.masked_fill(~allowed, -1e30), -1)
O = torch.einsum("bhgtk,bhkd->bhgtd", P, vf)
O.permute(0, 3, 1, 2, 4).reshape(B, T, -1).backward(dout.float())
for name, got, ref, ax in (("dk", dk, kf.grad, 2), ("dv", dv, vf.grad, 2), ("dq", dq, qf.grad, 3)):
    e = (got.float() - ref).abs()
    scale = ref.abs().max().item()
    tiles = [round(e.narrow(ax, t, min(32, T - t)).max().item() / scale, 4) for t in range(0, T, 32)]
    print(name, "per-tile rel err", tiles)
    if name != "dq":
        rows = (e.amax(dim=(0, 1, 3)) / scale)
        print("  worst rows", torch.topk(rows, 5).indices.tolist(), [round(x, 4) for x in torch.topk(rows, 5).values.tolist()])
