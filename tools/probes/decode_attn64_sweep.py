"""Per-row decode attention (decode_mfma_kernel) at the N = 8 rank's 64 rows in the rollout's form: groups of 8 sharing
512 prompt keys, 2 KV heads x 7 query heads, L cached keys, query position on the device, 8 cache copies rotated (cold),
graph-replayed. Every (waves, key-loop variant, key splits) forced. python tools/probes/decode_attn64_sweep.py [L,...]"""

import json
import sys

import torch

sys.path.insert(0, ".")
from dots.rl_amd import native  # noqa: E402

DEV, BF = "cuda", torch.bfloat16
B, group, Hkv, G, D, P, R = 64, 8, 2, 7, 64, 512, 256
Ls = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [520, 640, 767]
calls = 48
cap = P + R
g = torch.Generator(device=DEV).manual_seed(0)
caches = [(torch.randn(B, Hkv, cap, D, device=DEV, generator=g).to(BF),
           torch.randn(B, Hkv, cap // 32, D, 32, device=DEV, generator=g).to(BF)) for _ in range(8)]
valid = torch.ones(B, cap, dtype=torch.uint8, device=DEV)
q = torch.randn(B, Hkv, G, D, device=DEV, generator=g).to(BF)
outp = torch.empty(2 * 32 * Hkv * G * D, dtype=BF, device=DEV)
lib = native.lib()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def timed(L):
    qd = torch.full((1,), L - 1, dtype=torch.int64, device=DEV)

    def run():
        for i in range(calls):
            k, vt = caches[i % 8]
            native.decode_attention_vt(q, k, vt, valid, cap, outp, qpos_dev=qd, out_mbt=2, group=group, shared_keys=P)

    run()
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        graph.capture_begin()
        run()
        graph.capture_end()
    torch.cuda.synchronize()
    for _ in range(2):
        a.record()
        graph.replay()
        b.record()
        b.synchronize()
    return round(a.elapsed_time(b) * 1e3 / calls, 2), outp.clone()


for L in Ls:
    row = {"rows": B, "L": L}
    lib.drl_decode_attention_set_plan(0, 0)
    lib.drl_decode_attention_set_variant(0)
    row["planner"], ref = timed(L)
    for nw in (4, 8, 16):
        for var in (1, 2, 3, 4):
            for sp in (1, 2, 4):
                if sp > 1 and var != 2:
                    continue
                lib.drl_decode_attention_set_plan(nw, sp)
                lib.drl_decode_attention_set_variant(var)
                try:
                    t, out = timed(L)
                    row[f"nw{nw}_v{var}_s{sp}"] = t
                    d = (out.float() - ref.float()).abs().max().item()
                    if d > 0.05:
                        row[f"nw{nw}_v{var}_s{sp}_maxdiff"] = d
                except RuntimeError as e:
                    row[f"nw{nw}_v{var}_s{sp}"] = str(e)[:40]
    lib.drl_decode_attention_set_plan(0, 0)
    lib.drl_decode_attention_set_variant(0)
    print(json.dumps(row), flush=True)
