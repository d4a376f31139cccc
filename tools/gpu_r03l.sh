#!/bin/bash
# Counter passes (SQ, TCC) on drl_gemm at the fused shapes: where the K=896 / wgrad tiles lose time.
set -o pipefail
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r03l; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for shape in gate_up_fwd gate_up_wgrad gate_up_dgrad down_dgrad; do
  i=0
  for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" \
              "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU" \
              "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $pass -f csv -d "$OUT/${shape}_p$i" -o run -- python3 "$ROOT/tools/probes/sk_probe.py" $shape 4 > "$OUT/${shape}_p$i.log" 2>&1 || { tail -5 "$OUT/${shape}_p$i.log"; exit 1; }
  done
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/${shape}_t" -o run -- python3 "$ROOT/tools/probes/sk_probe.py" $shape 4 > "$OUT/${shape}_t.log" 2>&1 || { tail -5 "$OUT/${shape}_t.log"; exit 1; }
done
cd "$ROOT"
python3 - "$OUT" <<'PY'
import csv, glob, collections, sys, os
base = sys.argv[1]
for shape in ("gate_up_fwd", "gate_up_wgrad", "gate_up_dgrad", "down_dgrad"):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{base}/{shape}_p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "gemm_sk" in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur = []
    for f in glob.glob(f"{base}/{shape}_t/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "gemm_sk" in r["Kernel_Name"]:
                dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(shape, "us/launch", [round(d, 1) for d in dur])
    for k, v in sorted(acc.items()):
        print(f"   {k:28s} {sum(v) / len(v):16.1f}")
PY
find $OUT -name "*.csv" -size +5M -delete
