#!/bin/bash
# A/B of the C5 training step (res26-narrow, 4096 clips): kernel stats per variant of HONK_TRAIN_CONV.
set -e
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/trainab
mkdir -p "$OUT"
for v in ${VARIANTS:-m v}; do
  LIBP=$PWD/honk_amd/libhonk_hip.so; KV=$v
  if [ -f "$PWD/exp/_abl/$v/libhonk_hip.so" ]; then LIBP=$PWD/exp/_abl/$v/libhonk_hip.so; KV=m; fi
  HONK_LIB=$LIBP HONK_TRAIN_CONV=$KV timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT" -o $v --output-format csv -- \
    python3 bench.py --train --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/$v.log" 2>&1
  echo "== $v"; python3 exp/kstats.py "$OUT"/${v}_kernel_stats.csv
  grep -o '"value": [0-9.]*' "$OUT/$v.log" | head -1
done
