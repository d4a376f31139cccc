#!/bin/bash
# One MI355X job through gpurun: a chain of named steps, each under its own time limit; the chain stops at the
# first failure (a GPU fault, abort or time-limit kill ends the job, nothing is retried).
#   usage: bash tools/gpu.sh <tag> <step> [<step> ...]        (outputs under gpurun_out/<tag>/)
# steps:
#   tests                       the whole -m gpu suite
#   tests:<a>,<b>,...           the named pytest targets (files or node ids), -m gpu, verbose
#   bench[:<steps>[:<warmup>]]  the default bench line (no CPU baseline) + the last step's drl_gemm launch log
#   benchfull                   the driver's bench command (python bench.py, CPU baseline included)
#   benchfused                  the bench with model.use_fused_kernels=True
#   benchenv:<name>:<V=x>,...   the bench (5 steps, 2 warmup) with environment switches -> bench_<name>.json
#   bench64                     the per-rank workload of N = 8 (64 sequences) ; bench128 / bench256 likewise
#   benchx:<name>:<k=v>,<k=v>   the bench (5 steps, 2 warmup) with config overrides -> bench_<name>.json
#   profile                     rocprofv3 kernel stats of a 2-step bench + trace summary
#   pmc_gemm                    FETCH_SIZE / WRITE_SIZE passes over drl_gemm -> profiles/pmc_drl_gemm.json
#   pmc_flash                   two SQ counter passes over the fused attention kernels (tools/flash_quick.py)
#   ab:<lib>,<lib>,...          drl_gemm A/B over library builds (tools/gemm_ab.sh)
#   py:<script>[:<args>]        python -u <script> <args> (args split on ':')
set -o pipefail
TAG=${1:?tag}; shift
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp

run_tests() {  # $1 = log name, rest = pytest targets. Failed assertions (pytest rc 1) are reported and the chain goes
  # on; a crash, an interrupt or a time-limit kill (any other status) ends it.
  local log=$OUT/$1; shift
  timeout -k 10 900 python -u -m pytest "$@" -m gpu -q --timeout 300 --timeout-method thread > "$log" 2>&1
  local rc=$?
  tail -3 "$log"
  [ $rc = 0 ] && return 0
  grep -E "^FAILED|^ERROR|^BAD" "$log" | head -30
  [ $rc = 1 ] && return 0
  return 1
}

bench_rows() {  # $1 = sequences per step
  local b=$(( $1 / 8 )); local mini=$(( b / 2 < 4 ? 4 : b / 2 ))
  timeout -k 10 400 python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline --override data.train_batch_size=$b \
    actor_rollout_ref.actor.ppo_mini_batch_size=$mini > "$OUT/bench$1.json" 2> "$OUT/bench$1.err" \
    || { tail -20 "$OUT/bench$1.err"; return 1; }
  cut -c1-700 "$OUT/bench$1.json"
}

for step in "$@"; do
  echo "== $step"
  case "$step" in
    tests) run_tests tests.log tests || exit 1 ;;
    tests:*) IFS=',' read -ra T <<< "${step#tests:}"; run_tests "tests_$(date +%s).log" -v "${T[@]}" || exit 1 ;;
    bench|bench:*)
      IFS=':' read -ra A <<< "$step"; K=${A[1]:-5}; W=${A[2]:-2}
      timeout -k 10 500 python -u bench.py --steps "$K" --warmup "$W" --no-cpu-baseline \
        --launch-log "$OUT/gemm_launches.jsonl" > "$OUT/bench.json" 2> "$OUT/bench.err" \
        || { tail -20 "$OUT/bench.err"; exit 1; }
      cat "$OUT/bench.json" ;;
    benchfull)
      timeout -k 10 600 python -u bench.py > "$OUT/benchfull.json" 2> "$OUT/benchfull.err" \
        || { tail -20 "$OUT/benchfull.err"; exit 1; }
      cat "$OUT/benchfull.json" ;;
    benchfused)  # model.use_fused_kernels=True (A21 forward + the vocabulary-blocked HIP backward)
      timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline \
        --override actor_rollout_ref.model.use_fused_kernels=True > "$OUT/benchfused.json" 2> "$OUT/benchfused.err" \
        || { tail -20 "$OUT/benchfused.err"; exit 1; }
      cut -c1-900 "$OUT/benchfused.json" ;;
    benchx:*)
      IFS=':' read -ra A <<< "$step"; IFS=',' read -ra O <<< "${A[2]}"
      timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --override "${O[@]}" \
        > "$OUT/bench_${A[1]}.json" 2> "$OUT/bench_${A[1]}.err" || { tail -20 "$OUT/bench_${A[1]}.err"; exit 1; }
      cut -c1-900 "$OUT/bench_${A[1]}.json" ;;
    benchenv:*)  # benchenv:<name>:<VAR=val>,<VAR=val>: the bench (5 steps, 2 warmup) with environment switches
      IFS=':' read -ra A <<< "$step"; IFS=',' read -ra E <<< "${A[2]}"
      env "${E[@]}" timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline \
        --launch-log "$OUT/gemm_launches_${A[1]}.jsonl" > "$OUT/bench_${A[1]}.json" 2> "$OUT/bench_${A[1]}.err" \
        || { tail -20 "$OUT/bench_${A[1]}.err"; exit 1; }
      cut -c1-900 "$OUT/bench_${A[1]}.json" ;;
    bench64) bench_rows 64 || exit 1 ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 \
             || { tail -20 "$OUT/smoke.txt"; exit 1; }; tail -3 "$OUT/smoke.txt" ;;
    bench128) bench_rows 128 || exit 1 ;;
    bench256) bench_rows 256 || exit 1 ;;
    profile)
      DRL_TRACE_MARK=1 timeout -k 10 500 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o run -- python3 \
        "$ROOT/bench.py" --steps 2 --warmup 2 --no-cpu-baseline > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
      TR=$(find "$OUT/prof" -name "*kernel_trace.csv" | head -1)
      python3 tools/trace_summary.py "$TR" 30 > "$OUT/trace_summary.txt" || exit 1
      python3 tools/decode_gaps.py "$TR" > "$OUT/decode_step_512rows.txt" 2>&1 || true
      python3 - "$TR" "$OUT/kernel_trace_min.csv.gz" <<'PYEOF' || exit 1
import csv, gzip, sys
with gzip.open(sys.argv[2], "wt") as f:
    w = csv.writer(f)
    w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
    for r in csv.DictReader(open(sys.argv[1])):
        w.writerow([r["Kernel_Name"][:80], r["Start_Timestamp"], r["End_Timestamp"]])
PYEOF
      find "$OUT/prof" -name "*kernel_trace.csv" -delete
      head -40 "$OUT/trace_summary.txt" ;;
    pmc_gemm)
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 400 rocprofv3 --pmc $c --kernel-include-regex gemm_sk_kernel -f csv -d "$OUT/pmc_$c" -o p \
          -- python3 "$ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/pmc_$c.log" 2>&1 \
          || { tail -5 "$OUT/pmc_$c.log"; exit 1; }
      done
      python3 tools/pmc_traffic.py drl_gemm "$OUT/pmc_FETCH_SIZE" "$OUT/pmc_WRITE_SIZE" || exit 1
      cp profiles/pmc_drl_gemm.json "$OUT/"
      find "$OUT" -name "*.csv" -size +20M -delete ;;
    pmc_flash)
      i=0
      for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" \
                  "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_MFMA"; do
        i=$((i+1))
        timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-include-regex flash_ -f csv -d "$OUT/fpmc$i" -o p \
          -- python3 "$ROOT/tools/flash_quick.py" > "$OUT/fpmc$i.log" 2>&1 || { tail -5 "$OUT/fpmc$i.log"; exit 1; }
      done
      python3 tools/pmc_sq.py "$OUT/pmc_flash_sq.json" flash_fwd_kernel,flash_dq_kernel,flash_dkdv_kernel \
        "$OUT/fpmc1" "$OUT/fpmc2" || exit 1
      find "$OUT" -name "*.csv" -size +20M -delete ;;
    pmc_decattn)  # two SQ counter passes over the grouped decode attention (tools/probes/decode_attn_quick.py)
      i=0
      for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" \
                  "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU"; do
        i=$((i+1))
        timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-include-regex decode_group -f csv -d "$OUT/dpmc$i" -o p \
          -- python3 "$ROOT/tools/probes/decode_attn_quick.py" 640 48 > "$OUT/dpmc$i.log" 2>&1 || { tail -5 "$OUT/dpmc$i.log"; exit 1; }
      done
      python3 tools/pmc_sq.py "$OUT/pmc_decattn_sq.json" decode_group_kernel "$OUT/dpmc1" "$OUT/dpmc2" || exit 1
      find "$OUT" -name "*.csv" -size +20M -delete ;;
    pmc_shapes)  # FETCH_SIZE / WRITE_SIZE per update-pass shape class (tools/probes/pmc_shapes.py)
      timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d "$OUT/shp_t" -o t -- python3 "$ROOT/tools/probes/pmc_shapes.py" \
        > "$OUT/pmc_shapes.out" 2>&1 || { tail -5 "$OUT/pmc_shapes.out"; exit 1; }
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex gemm_sk_kernel -f csv -d "$OUT/shp_$c" -o p \
          -- python3 "$ROOT/tools/probes/pmc_shapes.py" > "$OUT/shp_$c.log" 2>&1 || { tail -5 "$OUT/shp_$c.log"; exit 1; }
      done
      python3 tools/pmc_shapes_summary.py "$OUT/pmc_shapes.out" "$OUT/shp_FETCH_SIZE" "$OUT/shp_WRITE_SIZE" \
        "$(find "$OUT/shp_t" -name "*kernel_trace.csv" | head -1)" > "$OUT/pmc_shapes.json" || exit 1
      find "$OUT" -name "*.csv" -size +20M -delete
      python3 -c "import json; [print(r['shape'], round(r['ratio'], 2), round(r.get('tflops', 0))) for r in json.load(open('$OUT/pmc_shapes.json'))['shapes']]" ;;
    ab:*)  # A/B of GEMM builds: ab:<lib1>,<lib2>,...
      IFS=',' read -ra L <<< "${step#ab:}"
      bash tools/gemm_ab.sh "$OUT" "${L[@]}" || exit 1 ;;
    py:*)
      IFS=':' read -ra A <<< "${step#py:}"
      timeout -k 10 600 python -u "${A[@]}" > "$OUT/$(basename "${A[0]}" .py).out" 2>&1; rc=$?
      tail -40 "$OUT/$(basename "${A[0]}" .py).out"; [ $rc = 0 ] || exit 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
