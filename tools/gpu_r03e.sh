#!/bin/bash
# GEMM backend A/B in the full step (roofline timer on the flash forward so the GEMM launches carry no events), then
# rocprofv3 kernel stats of each backend (stats only; the raw trace is deleted on the box).
set -o pipefail
OUT=gpurun_out/r03e; mkdir -p $OUT
summ() { grep '^{' $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); t=d['timing_s']; print('$2', round(d['value'],4), 'gen', round(t['gen'],3), 'logp', round(t['old_log_prob'],3), 'ref', round(t['ref'],3), 'upd', round(t['update_actor'],3), 'step', round(t['step'],3))"; }
for be in hip hipblaslt; do
  DRL_GEMM=$be timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --roofline-kernel drl_flash_attn_fwd > $OUT/bench_$be.log 2>&1 || { tail -30 $OUT/bench_$be.log; exit 1; }
  summ $OUT/bench_$be.log $be
done
DRL_CONCURRENT_WGRAD=0 timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --roofline-kernel drl_flash_attn_fwd > $OUT/bench_serial.log 2>&1 || { tail -30 $OUT/bench_serial.log; exit 1; }
summ $OUT/bench_serial.log hip_serial_wgrad
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for be in hip hipblaslt; do
  DRL_GEMM=$be timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_$be -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --roofline-kernel drl_flash_attn_fwd > $OUT/prof_$be.log 2>&1 || { tail -30 $OUT/prof_$be.log; exit 1; }
  f=$(find $OUT/prof_$be -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] || { find $OUT/prof_$be | head; exit 1; }
  cp $f $OUT/kernel_stats_$be.csv
  rm -rf $OUT/prof_$be
  python3 -c "
import csv
rows=list(csv.DictReader(open('$OUT/kernel_stats_$be.csv')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
tot=sum(float(r['TotalDurationNs']) for r in rows)
print('$be total kernel ms', round(tot/1e6,1))
for r in rows[:22]: print(f\"{float(r['TotalDurationNs'])/1e6:9.1f} ms {int(r['Calls']):7d} {float(r['AverageNs'])/1e3:9.1f}us  {r['Name'][:100]}\")
"
done
