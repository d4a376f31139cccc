#!/bin/bash
# HBM traffic per drl_gemm launch in the bench step (two PMC passes, FETCH_SIZE and WRITE_SIZE) -> pmc_drl_gemm.json
set -o pipefail
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_gemm; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex gemm_sk_kernel -f csv -d $OUT/f -o f -- python3 $ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/f.log 2>&1 || { tail -5 $OUT/f.log; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex gemm_sk_kernel -f csv -d $OUT/w -o w -- python3 $ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/w.log 2>&1 || { tail -5 $OUT/w.log; exit 1; }
cd $ROOT && python3 tools/pmc_traffic.py drl_gemm $OUT/f $OUT/w && cp profiles/pmc_drl_gemm.json $OUT/ && find $OUT -name "*.csv" -size +20M -delete
