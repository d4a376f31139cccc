#!/bin/bash
# In-situ GEMM shapes: kernel trace of one bench step per backend (drl_gemm serial wgrad / hipBLASLt), grouped by
# (kernel, grid); the raw trace is deleted on the box.
set -o pipefail
OUT=gpurun_out/r03f; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for be in hip hipblaslt; do
  DRL_CONCURRENT_WGRAD=0 DRL_GEMM=$be timeout -k 10 600 rocprofv3 --kernel-trace -f csv -d $OUT/tr_$be -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --roofline-kernel drl_flash_attn_fwd > $OUT/tr_$be.log 2>&1 || { tail -30 $OUT/tr_$be.log; exit 1; }
  f=$(find $OUT/tr_$be -name "*kernel_trace.csv" | head -1)
  [ -n "$f" ] || { find $OUT/tr_$be | head; exit 1; }
  python3 tools/trace_summary.py $f 16 14 > $OUT/shapes_$be.txt || exit 1
  rm -rf $OUT/tr_$be
  cat $OUT/shapes_$be.txt
done
