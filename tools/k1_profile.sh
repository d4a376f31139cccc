#!/bin/bash
# K1 evidence on one MI355X (through gpurun, repo root): GPU K1 parity tests, the 2^17..2^26 sweep, a rocprofv3
# kernel-trace summary of the 2^26 bench form and two PMC passes (FETCH_SIZE, WRITE_SIZE) per form.
# usage: bash tools/k1_profile.sh <tag>
set -o pipefail
TAG=${1:-k1}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "ppo or agg or kl" > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
timeout -k 10 200 python tools/kernel_bench.py --only k1 > "$OUT/sweep.jsonl" 2> "$OUT/sweep.err" || { tail "$OUT/sweep.err"; exit 1; }
cat "$OUT/sweep.jsonl"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT" || exit 1
for F in two_pass one_pass; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/stats_$F" -o run -- python bench.py --k1-only $F > "$OUT/stats_$F.log" 2>&1 || { tail "$OUT/stats_$F.log"; exit 1; }
  find "$OUT/stats_$F" -name "*kernel_trace.csv" -delete
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "ppo_loss_kernel|mask_pack_kernel" -f csv -d "$OUT/pmc_f_$F" -o f -- python bench.py --k1-only $F > "$OUT/pmc_f_$F.log" 2>&1 || { tail "$OUT/pmc_f_$F.log"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "ppo_loss_kernel|mask_pack_kernel" -f csv -d "$OUT/pmc_w_$F" -o w -- python bench.py --k1-only $F > "$OUT/pmc_w_$F.log" 2>&1 || { tail "$OUT/pmc_w_$F.log"; exit 1; }
  python tools/pmc_k1.py $F "$OUT/pmc_f_$F" "$OUT/pmc_w_$F" > "$OUT/pmc_$F.json" || exit 1
  cp profiles/pmc_drl_ppo_loss_fwd_bwd*.json "$OUT/"
  grep '^{' "$OUT/stats_$F.log"
done
