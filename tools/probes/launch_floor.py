"""Per-launch cost of short kernels inside a replayed HIP graph (the decode step is a dependent chain of them):
N launches of one kind captured back to back, wall time per launch over 50 replays. Kinds: a 1-element torch fill
(the trivial-kernel floor), dec_rmsnorm without partials, with 4 fp32 K-split partials (the down_proj seam), and the
same with the partials freshly written by a preceding fill (dirty in L2 at the boundary). Usage (GPU box):
python tools/probes/launch_floor.py [rows ...]
"""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dots.rl_amd import native  # noqa: E402


def per_launch_us(body, n):
    body()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        g.capture_begin()
        for _ in range(n):
            body()
        g.capture_end()
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(50):
        g.replay()
    b.record()
    b.synchronize()
    return round(a.elapsed_time(b) / 50 / n * 1e3, 2)


def main():
    rows = [int(r) for r in sys.argv[1:]] or [64, 512]
    H, dev, n = 896, "cuda", 200
    tiny = torch.zeros(1, device=dev)
    out = {"trivial_fill_1elem": per_launch_us(lambda: tiny.fill_(1.0), n)}
    for M in rows:
        x = torch.randn(M, H, device=dev)
        xo = torch.empty_like(x)
        w = torch.randn(H, device=dev)
        y = torch.empty(M, H, device=dev, dtype=torch.bfloat16)
        part = torch.randn(4, M, H, device=dev)
        r = {}
        r["rmsnorm_no_partials"] = per_launch_us(lambda: native.decode_rmsnorm(x, None, None, w, y, 1e-6), n)
        r["rmsnorm_4_partials"] = per_launch_us(lambda: native.decode_rmsnorm(x, part, xo, w, y, 1e-6), n)

        def dirty():
            part.fill_(0.5)
            native.decode_rmsnorm(x, part, xo, w, y, 1e-6)

        r["fill_partials_then_rmsnorm_pair"] = per_launch_us(dirty, n // 2)
        r["fill_partials_alone"] = per_launch_us(lambda: part.fill_(0.5), n)
        out[f"rows_{M}"] = r
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
