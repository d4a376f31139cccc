"""Recompute bench.py's drl_gemm roofline from a launch log (bench.py --launch-log): every timed drl_gemm call of one
bench step with its HIP-event interval, stream, work (2 M N K FLOP) and shape tag (M, N, K, a_layout, b_layout,
c_dtype, epilogue, dispatches).

  frac (per dispatch) = sum(work) / sum(call durations) / peak     (the rocprof view: mean kernel time x dispatches)
  frac_union          = sum(work) / |union of the call intervals| / peak   (side-stream weight gradients overlap)

Prints one JSON line with both and a per-shape table (calls, dispatches, total us, TFLOP/s), largest first.

  python tools/launch_log_summary.py profiles/r04_gemm_launches.jsonl
"""

import json
import sys
from collections import defaultdict

PEAK = 2500.0  # dense bf16 TFLOP/s (MI355X_MICROARCH.md)


def main(path):
    rows = [json.loads(line) for line in open(path)]
    work = sum(r["work"] for r in rows)
    dur = sum(r["end_us"] - r["start_us"] for r in rows)
    iv = sorted((r["start_us"], r["end_us"]) for r in rows)
    busy, cs, ce = 0.0, iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > ce:
            busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    disp = sum(r["tag"][7] for r in rows)
    ach, ach_u = work / dur / 1e6, work / busy / 1e6  # FLOP / us -> TFLOP/s
    shapes = defaultdict(lambda: [0, 0, 0.0, 0.0])
    for r in rows:
        M, N, K, al, bl, cdt, epi, nd = r["tag"]
        k = f"M{M} N{N} K{K} A{'KT'[al]} B{'KT'[bl]} {'f32' if cdt == 3 else 'bf16'} epi{epi}"
        s = shapes[k]
        s[0] += 1
        s[1] += nd
        s[2] += r["end_us"] - r["start_us"]
        s[3] += r["work"]
    print(json.dumps({"calls": len(rows), "dispatches": disp, "sum_call_us": round(dur, 1), "union_us": round(busy, 1),
                      "span_us": round(iv[-1][1] - iv[0][0], 1), "tflop": round(work / 1e12, 3),
                      "achieved_per_dispatch": round(ach, 1), "frac": round(ach / PEAK, 4),
                      "achieved_union": round(ach_u, 1), "frac_union": round(ach_u / PEAK, 4)}))
    for k, (n, nd, us, w) in sorted(shapes.items(), key=lambda kv: -kv[1][2]):
        print(f"{us:10.1f} us  {n:4d} calls {nd:4d} disp  {w / us / 1e6:7.1f} TF/s  {k}")


if __name__ == "__main__":
    main(sys.argv[1])
