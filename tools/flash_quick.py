"""Fused attention forward / backward timings at the fused-micro-batch shapes (update pass B = 32, log-prob pass
B = 80; T = 768, Qwen2.5-0.5B heads): one JSON line each. python tools/flash_quick.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import kernel_bench  # noqa: E402

for B in (32, 80):
    for r in kernel_bench.flash(B=B):
        r.pop("unfused_seconds", None)
        print(json.dumps(r), flush=True)
for r in kernel_bench.flash_bwd(B=32):
    print(json.dumps(r), flush=True)
