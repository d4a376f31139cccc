#!/bin/bash
# Remove-padding + drl_gemm tests, then the bench line and its rocprofv3 kernel summary.
set -o pipefail
OUT=gpurun_out/r03c; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_rmpad_gpu.py tests/test_gemm_sk_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/t.log 2>&1; rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" $OUT/t.log | tail -40; [ $rc = 0 ] || { tail -60 $OUT/t.log; exit 1; }
timeout -k 10 500 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['timing_s'], d['roofline'])"
DRL_CONCURRENT_WGRAD=0 timeout -k 10 500 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_serial.log 2>&1 || { tail -30 $OUT/bench_serial.log; exit 1; }
grep '^{' $OUT/bench_serial.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('serial wgrad', d['value'], d['ms_per_step'], d['timing_s'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/prof.log 2>&1 || { tail -30 $OUT/prof.log; exit 1; }
f=$(ls $OUT/prof/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] || f=$(ls $OUT/prof/run_kernel_stats.csv)
python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:25]: print(f\"{float(r['TotalDurationNs'])/1e6:9.1f} ms {int(r['Calls']):7d} {float(r['AverageNs'])/1e3:9.1f}us  {r['Name'][:110]}\")
"
