"""The 512-row decode lm_head on drl_gemm (M 512 x N 151936 x K 896: 1188 whole tiles = 4.64 rounds of 256 CUs),
graph-replayed with the weight cold in the MALL between calls (a 512 MiB scrub), under each decomposition / raster
group the tuning hook offers. python tools/probes/lm_head512.py"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402

from dots.rl_amd import native  # noqa: E402

lib = native.lib()
g = torch.Generator(device="cuda").manual_seed(0)
h = torch.randn(512, 896, device="cuda", generator=g).to(torch.bfloat16)
w = (torch.randn(151936, 896, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
out = torch.empty(512, 151936, device="cuda", dtype=torch.bfloat16)
scrub = torch.empty(512 * 2 ** 20, dtype=torch.uint8, device="cuda")
a_, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def run(tuning):
    lib.drl_gemm_set_sk_tuning(*tuning)
    native.gemm(h, native.LAYOUT_K, w, native.LAYOUT_K, 512, 151936, 896, out)
    torch.cuda.synchronize()
    ts = []
    for _ in range(12):
        scrub.fill_(1)
        a_.record()
        native.gemm(h, native.LAYOUT_K, w, native.LAYOUT_K, 512, 151936, 896, out)
        b_.record()
        b_.synchronize()
        ts.append(a_.elapsed_time(b_) * 1e3)
    ref = out.clone()
    lib.drl_gemm_set_sk_tuning(0, 0, 0, 0)
    return sorted(ts)[len(ts) // 2], ref


base_us, base = run((0, 0, 0, 0))
res = {"auto": round(base_us, 1)}
for name, tun in (("stream_k_tail", (0, 0, 1, 0)), ("group1", (0, 1, 0, 0)), ("group2", (0, 2, 0, 0)),
                  ("persistent_whole", (256, 0, 2, 0)), ("persistent_sk", (256, 0, 1, 0))):
    us, o = run(tun)
    res[name] = round(us, 1)
    res[name + "_same_bits"] = bool(torch.equal(o, base))
print(json.dumps(res), flush=True)
