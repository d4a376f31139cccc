# Round-end rehearsal on one MI355X (run through gpurun from the repo root): the GPU test suite, smoke(),
# then the round profile (bench line, rocprofv3 kernel stats, PMC traffic of the roofline kernel).
set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final/gputests.log 2>&1 || { tail -30 gpurun_out/final/gputests.log; exit 1; }
tail -2 gpurun_out/final/gputests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { tail -30 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
bash tools/gpu_profile.sh final drl_gemm_bf16_nt gemm_pp_kernel
