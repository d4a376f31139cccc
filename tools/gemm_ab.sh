#!/bin/bash
# A/B of drl_gemm builds (variants/*.so, same ABI; tools/build_variant.sh) on the config #2 pass shapes: one
# tools/gemm_sk_bench.py process per library. usage: bash tools/gemm_ab.sh <outdir> <lib.so> [<lib.so> ...]
set -o pipefail
OUT=$1; shift
mkdir -p "$OUT"
for lib in "$@"; do
  name=$(basename "$lib" .so)
  DRL_LIB_PATH=$(realpath "$lib") timeout -k 10 300 python -u tools/gemm_sk_bench.py --quick --no-lib \
    --rows 98304 196608 > "$OUT/ab_$name.jsonl" 2> "$OUT/ab_$name.err" || { tail -5 "$OUT/ab_$name.err"; exit 1; }
  echo "$name: $(wc -l < "$OUT/ab_$name.jsonl") shapes"
done
