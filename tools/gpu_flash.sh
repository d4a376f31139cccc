# Flash attention: parity tests, then forward / backward timing (tools/kernel_bench.py --only flash).
set -o pipefail
mkdir -p gpurun_out/flash
timeout -k 10 300 python -u -m pytest tests/test_layers_gpu.py tests/test_model_gpu.py tests/test_llama_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "flash or attention or logprob or rollout or backward" > gpurun_out/flash/t.log 2>&1; rc=$?; tail -3 gpurun_out/flash/t.log; [ $rc = 0 ] || exit 1
timeout -k 10 200 python tools/kernel_bench.py --only flash > gpurun_out/flash/bench.jsonl 2> gpurun_out/flash/bench.err || { tail gpurun_out/flash/bench.err; exit 1; }
cat gpurun_out/flash/bench.jsonl
