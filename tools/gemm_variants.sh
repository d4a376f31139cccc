#!/bin/bash
# GEMM A/B: libraries that differ only in gemm.hip's -D knobs (build here), then time them (GPU):
#   bash tools/gemm_variants.sh build ; (GPU) bash tools/gemm_variants.sh run
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/tools/probes/bin
VARS=${GVARS:-"base: nostore:-DDRL_GEMM_NOSTORE prio:-DDRL_GEMM_PRIO"}
if [ "$1" = build ]; then
  mkdir -p "$OUT"; rm -f "$OUT"/libg_*.so
  for v in $VARS; do
    name=${v%%:*}; flags=${v#*:}
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $flags -I"$ROOT/include" -I"$ROOT/dots.rl_amd/csrc" \
      -c "$ROOT/dots.rl_amd/csrc/gemm.hip" -o "/tmp/gvar_$name.o"
    objs=$(ls "$ROOT"/build/obj/*.o | grep -v "/gemm.hip.o")
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs "/tmp/gvar_$name.o" -o "$OUT/libg_$name.so"
  done
else
  mkdir -p "$ROOT/gpurun_out/gvar"
  for so in "$OUT"/libg_*.so; do
    n=$(basename "$so" .so)
    DOTSRL_AMD_LIB=$so timeout -k 10 200 python "$ROOT/tools/kernel_bench.py" --only gemm > "$ROOT/gpurun_out/gvar/$n.jsonl" 2>/dev/null
    python - "$ROOT/gpurun_out/gvar/$n.jsonl" "$n" <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
for r in rows:
    print(sys.argv[2], f"{r['layer']}@{r['M']}", "blas", round(r['hipblaslt_us']), "tiles", [round(r[f'tile{t}_us']) for t in range(1, 6)])
PY
  done
fi
