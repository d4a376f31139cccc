#!/bin/bash
# Build the native library with one csrc file replaced (A/B kernel experiments in one GPU call).
# Usage: tools/build_variant.sh <replacement.hip> <name-of-replaced-file.hip> <out.so>
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
cp "$ROOT"/dots.rl_amd/csrc/*.hip "$ROOT"/dots.rl_amd/csrc/*.h "$ROOT"/dots.rl_amd/csrc/*.cpp "$TMP"/
cp "$1" "$TMP/$2"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I"$ROOT/include" -I"$TMP" "$TMP"/*.hip "$TMP"/*.cpp -o "$3"
rm -rf "$TMP"
