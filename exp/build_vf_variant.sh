#!/bin/bash
# An experiment variant of libhonk_hip.so with res_vf.hip (the pair / last-layer kernels)
# recompiled under extra -D flags: exp/build_vf_variant.sh NAME "-DHONK_PAIR_PDM=1 ..."
#   -> exp/_var/libhonk_NAME.so (every other object from honk_amd/_build)
set -e
NAME=$1; DEFS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/exp/_var; mkdir -p "$OUT"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -I "$ROOT/include" \
  -mllvm -amdgpu-mfma-vgpr-form $DEFS -c "$ROOT/honk_amd/csrc/res_vf.hip" -o "$OUT/res_vf_$NAME.o"
OBJS="$OUT/res_vf_$NAME.o"
for f in runtime res cnn train mfcc head augment; do OBJS="$OBJS $ROOT/honk_amd/_build/$f.o"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libhonk_$NAME.so" $OBJS
echo "$OUT/libhonk_$NAME.so"
