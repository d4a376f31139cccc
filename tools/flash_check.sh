# flash attention: parity tests + forward staging-depth sweep + backward timing (run through gpurun)
set -o pipefail
mkdir -p gpurun_out/fa
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_layers_gpu.py -k flash > gpurun_out/fa/t.log 2>&1 || exit 1
timeout -k 10 200 python tools/kernel_bench.py --only flash > gpurun_out/fa/flash.jsonl 2>&1 || exit 1
timeout -k 10 100 python -c "
import sys; sys.argv=['x']; sys.path.insert(0,'tools')
import json, kernel_bench as kb
print(json.dumps(kb.flash_bwd()))" >> gpurun_out/fa/flash.jsonl 2>&1
