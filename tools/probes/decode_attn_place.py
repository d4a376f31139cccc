"""Decode attention placement: what the per-call floor of the decode attention is made of. The rollout's form (groups
of 8 sharing 512 prompt keys, 2 KV heads x 7 query heads, query position on the device, packed output), graph-replayed
48 calls, at 512 rows (prompt-group kernel) and 64 rows (per-row kernel): caches cold (4 copies rotated, > the 256 MB
MALL, every page's translation cold) against warm (one copy), the workgroup -> XCD map round-robin against XCD-contiguous
(drl_decode_group_set_plan), and a short cache (L = 64: the fixed cost). python tools/probes/decode_attn_place.py"""

import json
import sys

import torch

sys.path.insert(0, ".")
from dots.rl_amd import native  # noqa: E402

DEV, BF = "cuda", torch.bfloat16
group, Hkv, G, D, P, R = 8, 2, 7, 64, 512, 256
calls = 48
cap = P + R
lib = native.lib()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def timed(B, caches, valid, q, outp, L, shared):
    qd = torch.full((1,), L - 1, dtype=torch.int64, device=DEV)
    mbt = (B + 31) // 32

    def run():
        for i in range(calls):
            k, vt = caches[i % len(caches)]
            native.decode_attention_vt(q, k, vt, valid, cap, outp, qpos_dev=qd, out_mbt=mbt, group=group,
                                       shared_keys=shared)

    run()
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        graph.capture_begin()
        run()
        graph.capture_end()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        ev0.record()
        graph.replay()
        ev1.record()
        ev1.synchronize()
        best = min(best, ev0.elapsed_time(ev1) * 1e3 / calls)
    return round(best, 2), outp.clone()


for B in (512, 64):
    g = torch.Generator(device=DEV).manual_seed(B)
    caches = [(torch.randn(B, Hkv, cap, D, device=DEV, generator=g).to(BF),
               torch.randn(B, Hkv, cap // 32, D, 32, device=DEV, generator=g).to(BF)) for _ in range(4)]
    valid = torch.ones(B, cap, dtype=torch.uint8, device=DEV)
    q = torch.randn(B, Hkv, G, D, device=DEV, generator=g).to(BF)
    outp = torch.empty(((B + 31) // 32) * 32 * Hkv * G * D, dtype=BF, device=DEV)
    for L, shared in ((64, 32), (520, 512), (640, 512), (767, 512)):
        row = {"rows": B, "L": L}
        ref = None
        for xmap in (0, 1):
            lib.drl_decode_group_set_plan(0, xmap, 0)
            for name, cs in (("cold", caches), ("warm", caches[:1])):
                t, out = timed(B, cs, valid, q, outp, L, shared)
                row[f"{name}_x{xmap}"] = t
                if name == "cold":
                    if ref is None:
                        ref = out
                    elif not torch.equal(out, ref):
                        row[f"x{xmap}_differs"] = True
        lib.drl_decode_group_set_plan(0, 0, -1)
        print(json.dumps(row), flush=True)
    del caches
    torch.cuda.empty_cache()
