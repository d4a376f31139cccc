#!/bin/bash
# Round-3 checkpoint: full GPU suite, the default bench line, rocprofv3 kernel stats of the bench (stats kept, trace
# summarised per launch shape and deleted on the box).
set -o pipefail
OUT=gpurun_out/r03h; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gputests.log 2>&1; rc=$?; tail -4 $OUT/gputests.log; [ $rc = 0 ] || { grep -E "FAIL|Error" $OUT/gputests.log | head -20; exit 1; }
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log > $OUT/bench.json
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['timing_s'], d['roofline']['frac'], d['roofline']['mean_launch_us'], d['roofline_k1']['frac'], d['cpu_baseline']['value'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/prof.log 2>&1 || { tail -30 $OUT/prof.log; exit 1; }
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cp $f $OUT/kernel_stats.csv
t=$(find $OUT/prof -name "*kernel_trace.csv" | head -1); python3 tools/trace_summary.py $t 30 12 > $OUT/trace_summary.txt
rm -rf $OUT/prof
head -60 $OUT/trace_summary.txt | cut -c1-160
