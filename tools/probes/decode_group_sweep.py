"""Prompt-group decode attention (decode_group_kernel) at the N = 1 rollout's 512 rows in the rollout's form: groups of 8
sharing 512 prompt keys (cache rows 0..63 hold the prompts), 2 KV heads x 7 query heads, L cached keys, query position
on the device, packed output for the o_proj GEMM, 4 cache copies rotated (cold: 4 x 201 MB > the 256 MB MALL),
graph-replayed. Sweeps waves x rows per column tile x own-block schedule (drl_decode_group_set_plan: by block class /
balanced over the waves); every 8-wave plan's output must equal the default plan's (the same per-column arithmetic). python tools/probes/decode_group_sweep.py [L,...]"""

import json
import sys

import torch

sys.path.insert(0, ".")
from dots.rl_amd import native  # noqa: E402

DEV, BF = "cuda", torch.bfloat16
B, group, Hkv, G, D, P, R = 512, 8, 2, 7, 64, 512, 256
Ls = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [520, 580, 640, 700, 767]
calls = 48
cap = P + R
g = torch.Generator(device=DEV).manual_seed(0)
caches = [(torch.randn(B, Hkv, cap, D, device=DEV, generator=g).to(BF),
           torch.randn(B, Hkv, cap // 32, D, 32, device=DEV, generator=g).to(BF)) for _ in range(4)]
valid = torch.ones(B, cap, dtype=torch.uint8, device=DEV)
q = torch.randn(B, Hkv, G, D, device=DEV, generator=g).to(BF)
outp = torch.empty(16 * 32 * Hkv * G * D, dtype=BF, device=DEV)
lib = native.lib()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def timed(L):
    qd = torch.full((1,), L - 1, dtype=torch.int64, device=DEV)

    def run():
        for i in range(calls):
            k, vt = caches[i % len(caches)]
            native.decode_attention_vt(q, k, vt, valid, cap, outp, qpos_dev=qd, out_mbt=16, group=group,
                                       shared_keys=P)

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
        a.record()
        graph.replay()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) * 1e3 / calls)
    return round(best, 2), outp.clone()


plans = [(nw, rpt, bal) for nw in (4, 8) for rpt in (4, 2) for bal in (0, 1)]
for L in Ls:
    row = {"rows": B, "L": L}
    lib.drl_decode_attention_set_plan(0, 0)
    lib.drl_decode_group_set_plan(0, 0, -1)
    row["planner"], ref = timed(L)
    for nw, rpt, bal in plans:
        lib.drl_decode_attention_set_plan(nw, 0)
        lib.drl_decode_group_set_plan(rpt, 0, bal)
        key = f"nw{nw}_r{rpt}_{'bal' if bal else 'cls'}"
        try:
            t, out = timed(L)
            row[key] = t
            if nw == 8 and not torch.equal(out, ref):
                row[key + "_differs"] = (out.float() - ref.float()).abs().max().item()
        except RuntimeError as e:
            row[key] = str(e)[:40]
    lib.drl_decode_attention_set_plan(0, 0)
    lib.drl_decode_group_set_plan(0, 0, -1)
    print(json.dumps(row), flush=True)
