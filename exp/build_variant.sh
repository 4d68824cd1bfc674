#!/bin/bash
# Build an experiment variant of libhonk_hip.so from a (patched) copy of the csrc
# tree: exp/build_variant.sh NAME SRC_DIR [FILE]  ->  exp/_var/libhonk_NAME.so
# (FILE, default res, recompiled from SRC_DIR/FILE.hip; the other objects come from
# honk_amd/_build).  SRC_DIR's parent must hold include/ (a symlink to the repo's).
set -e
NAME=$1; SRC=$2; FILE=${3:-res}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/exp/_var; mkdir -p "$OUT"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -I "$ROOT/include" \
  ${HONK_VFLAGS} -c "$SRC/$FILE.hip" -o "$OUT/${FILE}_$NAME.o"
OBJS=""
for f in runtime res res_vf cnn train mfcc head augment; do
  if [ "$f" = "$FILE" ]; then OBJS="$OBJS $OUT/${FILE}_$NAME.o"; else OBJS="$OBJS $ROOT/honk_amd/_build/$f.o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libhonk_$NAME.so" $OBJS
echo "$OUT/libhonk_$NAME.so"
