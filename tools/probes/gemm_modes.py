"""drl_gemm schedule A/B at the update pass's 82144 rows, isolated and graph-replayed (10 calls): the split-K weight
gradients in slice-major vs tile-major workgroup order, and the gate_up gradient pair (input gradient M82144 N896
K9728 + weight gradient M9728 N896 K82144) concurrent on two streams vs in sequence, with the weight gradient as
whole tiles or stream-K. python tools/probes/gemm_modes.py"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402

from dots.rl_amd import native  # noqa: E402

T, H, I, NQ = 82144, 896, 4864, 1152
lib = native.lib()
a_, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
g = torch.Generator(device="cuda").manual_seed(0)
rnd = lambda *s: torch.randn(*s, device="cuda", generator=g).to(torch.bfloat16)  # noqa: E731


def gt(fn, calls=10):
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
    for _ in range(2):
        a_.record()
        gr.replay()
        b_.record()
        b_.synchronize()
    return round(a_.elapsed_time(b_) * 1e3 / calls, 1)


out = {}
for name, M, N in (("qkv_wgrad", NQ, H), ("o_wgrad", H, H), ("down_wgrad", H, I)):
    dy, x = rnd(T, M), rnd(T, N)
    gw = torch.zeros(M, N, device="cuda")
    ref = None
    for dbg in (0, 8):
        lib.drl_gemm_set_debug(dbg)
        out[f"{name}_{'tile' if dbg == 0 else 'slice'}_major_us"] = gt(lambda: native.linear_wgrad(gw, dy, x))
        gw.zero_()
        native.linear_wgrad(gw, dy, x)
        if ref is None:
            ref = gw.clone()
        else:
            out[f"{name}_orders_bit_identical"] = bool(torch.equal(ref, gw))
    lib.drl_gemm_set_debug(0)
    del dy, x, gw
dgu, w, h2 = rnd(T, 2 * I), rnd(2 * I, H) * 0.05, rnd(T, H)
gw = torch.zeros(2 * I, H, device="cuda")
side = torch.cuda.Stream()


def pair(concurrent):
    if concurrent:
        main = torch.cuda.current_stream()
        side.wait_stream(main)
        with torch.cuda.stream(side):
            native.linear_wgrad(gw, dgu, h2, ws_slot=1)
        native.linear_dgrad(dgu, w)
        main.wait_stream(side)
    else:
        native.linear_wgrad(gw, dgu, h2)
        native.linear_dgrad(dgu, w)


out["gate_up_dgrad_us"] = gt(lambda: native.linear_dgrad(dgu, w))
out["gate_up_wgrad_whole_us"] = gt(lambda: native.linear_wgrad(gw, dgu, h2))
out["gate_up_pair_concurrent_us"] = gt(lambda: pair(True))
out["gate_up_pair_sequential_us"] = gt(lambda: pair(False))
for minit in (0, 4, 8):
    lib.drl_gemm_set_sk_tuning(0, 0, 1, minit)
    out[f"gate_up_wgrad_streamk_min{minit}_us"] = gt(lambda: native.linear_wgrad(gw, dgu, h2))
lib.drl_gemm_set_sk_tuning(0, 0, 0, 0)
print(json.dumps(out), flush=True)
