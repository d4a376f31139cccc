#!/bin/bash
# A/B of library builds on one probe script in one GPU call: rounds x (each library in turn), alternating, so box
# drift hits every build alike. usage: bash tools/probes/ab_run.sh <rounds> "<python script + args>" <lib.so> ...
set -o pipefail
ROUNDS=$1; CMD=$2; shift 2
for r in $(seq 1 "$ROUNDS"); do
  for lib in "$@"; do
    out=$(DRL_LIB_PATH=$(realpath "$lib") timeout -k 10 120 python -u $CMD 2>/dev/null) || { echo "FAIL $lib"; exit 1; }
    echo "round $r $(basename "$lib" .so): $out"
  done
done
