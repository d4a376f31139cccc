set -o pipefail
mkdir -p gpurun_out/k4
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_decode_gemm_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "sampl or select or top_p or rollout" > gpurun_out/k4/t.log 2>&1; rc=$?; tail -5 gpurun_out/k4/t.log; [ $rc = 0 ] || exit 1
timeout -k 10 120 python tools/kernel_bench.py --only k2 > gpurun_out/k4/k2.jsonl 2>&1 || exit 1
cat gpurun_out/k4/k2.jsonl
