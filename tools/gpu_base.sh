#!/bin/bash
# Round baseline on one MI355X: full -m gpu suite, default bench line, rocprofv3 kernel stats of the bench.
# usage: bash tools/gpu_base.sh <tag>
set -o pipefail
TAG=${1:-r02}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gputests.log" 2>&1 \
  || { tail -40 "$OUT/gputests.log"; exit 1; }
tail -2 "$OUT/gputests.log"
timeout -k 10 400 python bench.py > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
grep '^{' "$OUT/bench.log"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT" || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/stats" -o run -- python bench.py --no-cpu-baseline > "$OUT/stats.log" 2>&1 || { tail -20 "$OUT/stats.log"; exit 1; }
TR=$(find "$OUT/stats" -name "*kernel_trace.csv" | head -1)
python tools/trace_summary.py "$TR" 25 > "$OUT/trace_summary.txt" 2>&1 || true
find "$OUT/stats" -name "*kernel_trace.csv" -delete
head -30 "$OUT/trace_summary.txt"
