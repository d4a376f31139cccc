"""Decode attention under prompt groups (decode_group_kernel) (the rollout's config #2 form: 512 rows in groups of 8, 2 KV heads x 7 query
heads, 512 shared prompt keys, 1..256 response keys): every (waves, variant, splits) plan of drl_decode_attention_vt
over cold caches (copies rotated past the MALL), outputs checked identical to the automatic plan.

  python tools/probes/decode_group_sweep.py [B]    -> one JSON line per (L, plan); B < 512: the per-row plans"""

import json
import sys

import torch

sys.path.insert(0, ".")
from dots.rl_amd import native  # noqa: E402

DEV, BF = "cuda", torch.bfloat16
B, group, Hkv, G, D, P, R = int(sys.argv[1]) if len(sys.argv) > 1 else 512, 8, 2, 7, 64, 512, 256
cap = P + R
lib = native.lib()
g = torch.Generator(device=DEV).manual_seed(0)
ncopy = 8  # 8 x 2 x 512 x 768 x 64 x 2 x 2 B = 1.6 GB of caches: each call reads a cold copy
nb = cap // 32
caches = []
for c in range(ncopy):
    k = torch.randn(B, Hkv, cap, D, device=DEV, generator=g).to(BF)
    vt = torch.randn(B, Hkv, nb, D, 32, device=DEV, generator=g).to(BF)
    caches.append((k, vt))
valid = torch.ones(B, cap, dtype=torch.uint8, device=DEV)
q = torch.randn(B, Hkv, G, D, device=DEV, generator=g).to(BF)
# decode_group_kernel at its default 8 waves and forced 2 / 4 / 16 (the per-row kernel's plans no longer apply
# to grouped calls; its numbers before the grouped kernel: profiles/r04_decode_group_perrow.jsonl)
plans = [(0, 0, 0), (2, 0, 0), (4, 0, 0), (16, 0, 0)]
if B < 512:  # below the grouped kernel's threshold the per-row kernel runs: its (waves, variant, splits) plans
    plans = [(0, 0, 0)] + [(w, v, sp) for w in (2, 4, 8, 16) for v in (0, 1, 2, 3, 4) for sp in (1, 2, 4)]
for L in (P + 32, P + 128, P + 256):
    outs = {}
    for (w, v, s) in plans:
        lib.drl_decode_attention_set_plan(w, s)
        lib.drl_decode_attention_set_variant(v)
        out = torch.empty_like(q)
        i = [0]

        def call():
            k, vt = caches[i[0] % ncopy]
            i[0] += 1
            native.decode_attention_vt(q, k, vt, valid, L, out, group=group, shared_keys=P)

        try:
            for _ in range(3):
                call()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ts = []
            for _ in range(5):
                a.record()
                for _ in range(16):
                    call()
                b.record()
                b.synchronize()
                ts.append(a.elapsed_time(b) * 1e3 / 16)
            ts.sort()
            i[0] = 0
            call()
            same = None
            if (0, 0, 0) in outs:
                same = bool(torch.equal(out, outs[(0, 0, 0)]))
            else:
                outs[(w, v, s)] = out.clone()
            print(json.dumps(dict(L=L, waves=w, variant=v, splits=s, us=round(ts[2], 2), us_min=round(ts[0], 2),
                                  same_as_auto=same)), flush=True)
        except RuntimeError as e:
            print(json.dumps(dict(L=L, waves=w, variant=v, splits=s, error=str(e)[:120])), flush=True)
lib.drl_decode_attention_set_plan(0, 0)
lib.drl_decode_attention_set_variant(0)
# the rollout's form, taken apart: (b) host query position sweeping 512..767 with the capacity as the length
# argument; (c) the position in device memory rewritten before each call (a fill kernel in the loop); (d) the
# position in device memory, fixed; packed output for the o_proj GEMM in (c) / (d) as in the rollout
qd = torch.full((1,), P + 127, dtype=torch.int64, device=DEV)
outp = torch.empty(16 * 32 * Hkv * G * D, dtype=BF, device=DEV)


def timed(call, n=64):
    for _ in range(3):
        call()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        call()
    b.record()
    b.synchronize()
    return round(a.elapsed_time(b) * 1e3 / n, 2)


ctr = [0]


def form(kind):
    def call():
        k, vt = caches[ctr[0] % ncopy]
        ctr[0] += 1
        if kind == "b":
            native.decode_attention_vt(q, k, vt, valid, cap, torch.empty_like(q), qpos=P + (ctr[0] * 37) % R,
                                       group=group, shared_keys=P)
        elif kind == "c":
            qd.fill_(P + (ctr[0] * 37) % R)
            native.decode_attention_vt(q, k, vt, valid, cap, outp, qpos_dev=qd, out_mbt=16, group=group,
                                       shared_keys=P)
        elif kind == "fill":
            qd.fill_(P + (ctr[0] * 37) % R)
        else:
            native.decode_attention_vt(q, k, vt, valid, cap, outp, qpos_dev=qd, out_mbt=16, group=group,
                                       shared_keys=P)
    return call


for kind in ("b", "c", "d", "fill"):
    print(json.dumps(dict(form=kind, us=timed(form(kind)))), flush=True)
qd.fill_(P + 127)
print(json.dumps(dict(form="d_L640", us=timed(form("d")))), flush=True)
