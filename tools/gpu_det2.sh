#!/bin/bash
set -o pipefail
OUT=gpurun_out/det2; mkdir -p $OUT
timeout -k 10 300 python tools/probes/det_probe2.py > $OUT/det.log 2>&1 || { tail -30 $OUT/det.log; exit 1; }
grep -E '^run|^   ' $OUT/det.log | head -60
