# K1 A/B in one GPU call: variant libraries built by tools/build_variant.sh (build/var/lib_<name>.so),
# plus the no-math streaming ceiling of the same box (tools/hbm_probe.hip).
set -e
cd /root/repo
timeout -k 10 120 ./build/hbm_probe > gpurun_out/k1var_probe.jsonl 2>&1
for n in ${K1VARS:-pf0_w4 pf1_w4}; do
  DOTSRL_AMD_LIB=build/var/lib_$n.so timeout -k 10 200 python tools/kernel_bench.py --only k1 > gpurun_out/k1var_$n.jsonl 2>/dev/null
done
