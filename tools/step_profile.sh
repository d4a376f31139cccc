# Kernel-time breakdown of the bench step on one MI355X (run through gpurun from the repo root):
#   rocprofv3 kernel stats + per-shape summary of the top kernels. Usage: bash tools/step_profile.sh <tag> [bench args]
set -o pipefail
TAG=${1:-prof}; shift
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT" || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o run -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline "$@" > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
python3 tools/trace_summary.py $(find "$OUT/prof" -name "*kernel_trace.csv" | head -1) 30 > "$OUT/trace_summary.txt" || exit 1
find "$OUT/prof" -name "*kernel_trace.csv" -delete
grep '^{' "$OUT/prof.log" | head -1 | cut -c1-600
