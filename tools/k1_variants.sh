#!/bin/bash
# K1 A/B: build libraries that differ only in ppo_loss.hip's -D knobs (run here, on the CPU), then time each
# on the GPU: bash tools/k1_variants.sh build ; (GPU) bash tools/k1_variants.sh run
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/tools/probes/bin
VARS=${K1VARS:-"u2p1w2:-DDRL_K1_U=2 -DDRL_K1_PIPE=1 -DDRL_K1_WG_PER_CU=2 u1p1w2:-DDRL_K1_U=1 -DDRL_K1_PIPE=1 -DDRL_K1_WG_PER_CU=2 u2p0w2:-DDRL_K1_U=2 -DDRL_K1_PIPE=0 -DDRL_K1_WG_PER_CU=2 u4p0w2:-DDRL_K1_U=4 -DDRL_K1_PIPE=0 -DDRL_K1_WG_PER_CU=2 u2p1w4:-DDRL_K1_U=2 -DDRL_K1_PIPE=1 -DDRL_K1_WG_PER_CU=4 u1p1w4:-DDRL_K1_U=1 -DDRL_K1_PIPE=1 -DDRL_K1_WG_PER_CU=4"}
if [ "$1" = build ]; then
  mkdir -p "$OUT"
  IFS=' ' read -ra parts <<< "$VARS"
  name=""; flags=""
  build_one() {
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $2 -I"$ROOT/include" -I"$ROOT/dots.rl_amd/csrc" \
      -c "$ROOT/dots.rl_amd/csrc/ppo_loss.hip" -o "/tmp/k1var_$1.o"
    objs=$(ls "$ROOT"/build/obj/*.o | grep -v ppo_loss)
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs "/tmp/k1var_$1.o" -o "$OUT/lib_$1.so"
  }
  for tok in "${parts[@]}"; do
    if [[ "$tok" == *:* ]]; then
      [ -n "$name" ] && build_one "$name" "$flags"
      name=${tok%%:*}; flags=${tok#*:}
    else
      flags="$flags $tok"
    fi
  done
  [ -n "$name" ] && build_one "$name" "$flags"
else
  mkdir -p "$ROOT/gpurun_out/k1var"
  for so in "$OUT"/lib_*.so; do
    n=$(basename "$so" .so)
    DOTSRL_AMD_LIB=$so timeout -k 10 100 python "$ROOT/bench.py" --k1-only one_pass > "$ROOT/gpurun_out/k1var/$n.one.json"
    DOTSRL_AMD_LIB=$so timeout -k 10 100 python "$ROOT/bench.py" --k1-only two_pass > "$ROOT/gpurun_out/k1var/$n.two.json"
    echo "$n one $(python -c "import json;d=json.load(open('$ROOT/gpurun_out/k1var/$n.one.json'));print(round(d['frac'],4))") two $(python -c "import json;d=json.load(open('$ROOT/gpurun_out/k1var/$n.two.json'));print(round(d['frac'],4))")"
  done
fi
