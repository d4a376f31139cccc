# SQ / TCC counter passes over tools/probes/gemm_probe.py for the ping-pong GEMM (one rocprofv3 --pmc run per
# pass; run through gpurun). Usage: bash tools/gemm_pmc.sh <shape>
set -o pipefail
SHAPE=${1:-lm_head}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/gpmc_$SHAPE
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" \
            "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pass -f csv -d "$OUT/p$i" -o run -- python3 "$ROOT/tools/probes/gemm_probe.py" $SHAPE 5 > "$OUT/p$i.log" 2>&1 || { tail -5 "$OUT/p$i.log"; exit 1; }
done
cd "$ROOT"
python3 - "$OUT" <<'PY'
import csv, glob, collections, sys
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "gemm_pp" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(f"{k:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
PY
