mkdir -p gpurun_out/sqg && export TMPDIR=/tmp && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex gemm_sk_kernel -f csv -d gpurun_out/sqg/p1 -o p -- python3 tools/probes/sk_probe.py gate_up_fwd 5 > gpurun_out/sqg/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVES --kernel-include-regex gemm_sk_kernel -f csv -d gpurun_out/sqg/p2 -o p -- python3 tools/probes/sk_probe.py gate_up_fwd 5 > gpurun_out/sqg/p2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex gemm_sk_kernel -f csv -d gpurun_out/sqg/p3 -o p -- python3 tools/probes/sk_probe.py down_fwd 5 > gpurun_out/sqg/p3.log 2>&1 && \
python3 tools/pmc_sq.py gpurun_out/sqg/gate_up_fwd_sq.json gemm_sk_kernel gpurun_out/sqg/p1 gpurun_out/sqg/p2 && \
python3 tools/pmc_sq.py gpurun_out/sqg/down_fwd_sq.json gemm_sk_kernel gpurun_out/sqg/p3 && \
find gpurun_out/sqg -name "*.csv" -size +5M -delete
