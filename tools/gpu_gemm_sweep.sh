# Hand-written GEMM tile sweep vs hipBLASLt (tools/kernel_bench.py --only gemm) and its parity tests.
set -o pipefail
mkdir -p gpurun_out/gemm
timeout -k 10 200 python -u -m pytest tests/test_gemm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gemm/t.log 2>&1; rc=$?; tail -3 gpurun_out/gemm/t.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python tools/kernel_bench.py --only gemm > gpurun_out/gemm/sweep.jsonl 2> gpurun_out/gemm/sweep.err || { tail gpurun_out/gemm/sweep.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/gemm/sweep.jsonl'):
    r=json.loads(l); ks=sorted(k for k in r if k.endswith('_TF'))
    print(r['layer'], r['M'], ' '.join(f'{k[:-3]}={r[k]:.0f}' for k in ks))
"
