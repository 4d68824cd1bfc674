#!/bin/bash
# Build an experiment variant of libhonk_hip.so from a (patched) copy of the csrc
# tree: exp/build_variant.sh NAME SRC_DIR  ->  exp/_var/libhonk_NAME.so
# (res.hip recompiled from SRC_DIR; the other objects come from honk_amd/_build).
set -e
NAME=$1; SRC=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/exp/_var; mkdir -p "$OUT"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -I "$ROOT/include" \
  -c "$SRC/res.hip" -o "$OUT/res_$NAME.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libhonk_$NAME.so" "$OUT/res_$NAME.o" \
  "$ROOT/honk_amd/_build/runtime.o" "$ROOT/honk_amd/_build/cnn.o" "$ROOT/honk_amd/_build/train.o" \
  "$ROOT/honk_amd/_build/mfcc.o"
echo "$OUT/libhonk_$NAME.so"
