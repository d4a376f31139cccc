#!/bin/bash
# Round profile on one MI355X (run through gpurun from the repo root):
#   bench line, rocprofv3 kernel stats of the same command, two PMC passes for the roofline kernel.
# Usage: bash tools/gpu_profile.sh <round-tag> [roofline-kernel-symbol] [kernel-name-regex]
set -o pipefail
TAG=${1:-r01}
SYM=${2:-drl_flash_attn_fwd}
RX=${3:-flash_fwd_kernel}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT" || exit 1
timeout -k 10 600 python bench.py --roofline-kernel "$SYM" > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
grep '^{' "$OUT/bench.log" > "$OUT/bench.json"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/stats" -o run -- python bench.py --roofline-kernel "$SYM" > "$OUT/stats.log" 2>&1 || { tail -20 "$OUT/stats.log"; exit 1; }
grep '^{' "$OUT/stats.log" > "$OUT/stats_bench.json"
find "$OUT/stats" -name "*kernel_trace.csv" -delete
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" -f csv -d "$OUT/pmc_f" -o f -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --roofline-kernel "$SYM" > "$OUT/pmc_f.log" 2>&1 || { tail -20 "$OUT/pmc_f.log"; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" -f csv -d "$OUT/pmc_w" -o w -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --roofline-kernel "$SYM" > "$OUT/pmc_w.log" 2>&1 || { tail -20 "$OUT/pmc_w.log"; exit 1; }
python tools/pmc_traffic.py "$SYM" "$OUT/pmc_f" "$OUT/pmc_w" > "$OUT/pmc.json" && cp "profiles/pmc_$SYM.json" "$OUT/" || exit 1
find "$OUT" -name "*counter_collection.csv" -size +20M -delete
cat "$OUT/bench.json"
