# Round check through gpurun: whole -m gpu suite, a short default bench, then the 512-row step profile.
# usage: bash tools/gpu_round_check.sh <tag>
set -o pipefail
TAG=${1:-rc}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/gputests.log 2>&1
tail -3 gpurun_out/$TAG/gputests.log
grep -q " passed" gpurun_out/$TAG/gputests.log && ! grep -q " failed\|[0-9] error" gpurun_out/$TAG/gputests.log || exit 1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/b512.json 2> gpurun_out/$TAG/b512.err || exit 1
cut -c1-400 gpurun_out/$TAG/b512.json
bash tools/step_profile.sh ${TAG}p512
