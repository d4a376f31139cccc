"""drl_gemm A/B of the half-width last tile column (N % 256 in (0, 128]: the N = 896 / 1152 outputs of the update and
log-prob passes) against the full-width tiles it replaces (drl_gemm_set_debug bit 32), isolated and graph-replayed,
at the pass shapes (82144 / 164288 rows). Interleaved rounds, median per arm. python tools/probes/half_tile_ab.py"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402

from dots.rl_amd import native  # noqa: E402

lib = native.lib()
g = torch.Generator(device="cuda").manual_seed(0)
rnd = lambda *s: torch.randn(*s, device="cuda", generator=g).to(torch.bfloat16)  # noqa: E731
a_, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def graph_us(fn, calls=10):
    fn()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        gr.capture_begin()
        for _ in range(calls):
            fn()
        gr.capture_end()
    torch.cuda.synchronize()
    gr.replay()
    a_.record()
    gr.replay()
    b_.record()
    b_.synchronize()
    return a_.elapsed_time(b_) * 1e3 / calls


H, I, NQ = 896, 4864, 1152
cases = []
for T in (82144, 164288):
    x, w_o, w_d, w_q = rnd(T, H), rnd(H, H) * 0.05, rnd(H, I) * 0.05, rnd(NQ, H) * 0.05
    a, bq = rnd(T, I), rnd(NQ)
    cases += [(f"o_fwd_{T}", lambda x=x, w=w_o: native.linear_fwd(x, w)),
              (f"down_fwd_{T}", lambda a=a, w=w_d: native.linear_fwd(a, w)),
              (f"qkv_fwd_bias_{T}", lambda x=x, w=w_q, b=bq: native.linear_fwd(x, w, bias=b))]
T = 82144
dy_o, dy_q, dy_gu = rnd(T, H), rnd(T, NQ), rnd(T, 2 * I)
w_o, w_q, w_gu, x = rnd(H, H) * 0.05, rnd(NQ, H) * 0.05, rnd(2 * I, H) * 0.05, rnd(T, H)
gw = torch.zeros(2 * I, H, device="cuda")
cases += [("o_dgrad_82144", lambda: native.linear_dgrad(dy_o, w_o)),
          ("qkv_dgrad_82144", lambda: native.linear_dgrad(dy_q, w_q)),
          ("gate_up_dgrad_82144", lambda: native.linear_dgrad(dy_gu, w_gu)),
          ("gate_up_wgrad_82144", lambda: native.linear_wgrad(gw, dy_gu, x))]
res = {n: {"half": [], "full": []} for n, _ in cases}
for rnd_i in range(3):
    for n, fn in cases:
        for arm, dbg in (("half", 0), ("full", 32)):
            lib.drl_gemm_set_debug(dbg)
            res[n][arm].append(graph_us(fn))
lib.drl_gemm_set_debug(0)
out = {}
for n, r in res.items():
    h, f = sorted(r["half"])[1], sorted(r["full"])[1]
    out[n] = {"half_us": round(h, 1), "full_us": round(f, 1), "ratio": round(h / f, 3)}
    print(json.dumps({n: out[n]}), flush=True)
