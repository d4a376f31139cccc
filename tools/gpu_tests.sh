# GPU parity tests through gpurun: named test files first (verbose), then optionally the whole -m gpu suite (ALL=1).
# usage: [ALL=1] bash tools/gpu_tests.sh [pytest args...]
set -o pipefail
OUT=gpurun_out/t
mkdir -p $OUT
if [ $# -gt 0 ]; then
  timeout -k 10 400 python -u -m pytest "$@" -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/first.log 2>&1 \
    || { tail -60 $OUT/first.log; exit 1; }
  grep -E "PASSED|FAILED|ERROR" $OUT/first.log | tail -25
fi
if [ "${ALL:-0}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/all.log 2>&1 \
    || { tail -40 $OUT/all.log; exit 1; }
  tail -2 $OUT/all.log
fi
