"""A short workload for counter passes over the grouped decode attention (decode_group_kernel) in the rollout's form
at 512 rows: groups of 8, 2 KV heads x 7 query heads, 512 shared prompt keys, L cached keys (default 640), the query
position in device memory, cold caches (8 copies rotated). python tools/probes/decode_attn_quick.py [L[,L...]] [calls]"""

import sys

import torch

sys.path.insert(0, ".")
from dots.rl_amd import native  # noqa: E402

DEV, BF = "cuda", torch.bfloat16
import os  # noqa: E402

B = int(os.environ.get("DEC_B", "512"))  # 64: the N = 8 rank's rows (the per-row kernel)
group, Hkv, G, D, P, R = 8, 2, 7, 64, 512, 256
Ls = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [640]
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 48
cap = P + R
g = torch.Generator(device=DEV).manual_seed(0)
caches = [(torch.randn(B, Hkv, cap, D, device=DEV, generator=g).to(BF),
           torch.randn(B, Hkv, cap // 32, D, 32, device=DEV, generator=g).to(BF)) for _ in range(8)]
valid = torch.ones(B, cap, dtype=torch.uint8, device=DEV)
q = torch.randn(B, Hkv, G, D, device=DEV, generator=g).to(BF)
outp = torch.empty(16 * 32 * Hkv * G * D, dtype=BF, device=DEV)
mbt = (B + 31) // 32
if os.environ.get("DEC_NW"):  # forced waves per workgroup (drl_decode_attention_set_plan)
    native.lib().drl_decode_attention_set_plan(int(os.environ["DEC_NW"]), 0)
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
res = []
# the calls are captured in one HIP graph and replayed (the rollout's form): eager launches from Python are
# host-bound at these sizes (~11 us per call whatever the kernel does)
for L in Ls:
    qd = torch.full((1,), L - 1, dtype=torch.int64, device=DEV)

    def run():
        for i in range(calls):
            k, vt = caches[i % 8]
            native.decode_attention_vt(q, k, vt, valid, cap, outp, qpos_dev=qd, out_mbt=mbt, group=group, shared_keys=P)

    run()  # workspaces allocated outside the capture
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        graph.capture_begin()
        run()
        graph.capture_end()
    torch.cuda.synchronize()
    for rep in range(2):
        a.record()
        graph.replay()
        b.record()
        b.synchronize()
    res.append(f"L={L}: {a.elapsed_time(b) * 1e3 / calls:.2f}")
print(" ".join(res), "us per call (graph replay)")
