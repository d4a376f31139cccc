set -o pipefail
mkdir -p gpurun_out/r4p && cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r4p/prof -o run -- python3 tools/probes/flash_ab.py run prof > gpurun_out/r4p/prof.log 2>&1 || { tail -5 gpurun_out/r4p/prof.log; exit 1; }
find gpurun_out/r4p/prof -name '*kernel_stats.csv' -exec cp {} gpurun_out/r4p/stats.csv \;
find gpurun_out/r4p/prof -name '*kernel_trace.csv' -delete
cut -d, -f1-4 gpurun_out/r4p/stats.csv | head -12
