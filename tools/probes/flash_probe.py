"""Flash attention forward at the update micro-batch shape (B=8, T=768, 14/2 heads, D=64), a few launches:
the program rocprofv3 --pmc passes profile (tools/flash_pmc.sh)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dots.rl_amd import native  # noqa: E402

B, Hkv, G, D, T = 8, 2, 7, 64, 768
dev = "cuda"
q = torch.randn(B, Hkv, G, T, D, device=dev, dtype=torch.bfloat16)
k = torch.randn(B, Hkv, T, D, device=dev, dtype=torch.bfloat16)
vt = torch.randn(B, Hkv, D, T, device=dev, dtype=torch.bfloat16)
valid = torch.ones(B, T, dtype=torch.uint8, device=dev)
out = torch.empty(B, T, Hkv * G * D, device=dev, dtype=torch.bfloat16)
lse = torch.empty(B, Hkv, G, T, device=dev)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
    native.flash_attn_fwd(q, k, vt, valid, out, lse=lse)
torch.cuda.synchronize()
