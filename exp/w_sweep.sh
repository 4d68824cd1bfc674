#!/bin/bash
# Timing sweep of the weight-stationary res kernel: ablation builds (exp/ablate_w.py)
# and batch-chunk sizes, one rocprofv3 kernel-stats pass each (res15 bf16x3).
set -e
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/wsweep
mkdir -p "$OUT"
ARGS="bench.py --batch 16384 --steps 2 --warmup 1 --no-cpu-baseline --no-configs --no-alt"
for v in ${VARIANTS:-base nostore nores nodma noepi mfma}; do
  LIBP=$PWD/exp/_abl/$v/libhonk_hip.so; [ "$v" = cur ] && LIBP=$PWD/honk_amd/libhonk_hip.so
  HONK_LIB=$LIBP timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT" -o $v \
    --output-format csv -- python3 $ARGS > "$OUT/$v.log" 2>&1
  echo "== $v"; python3 exp/kstats.py "$OUT"/$v*_kernel_stats.csv
done
for c in ${CHUNKS:-}; do
  HONK_RES_CHUNK=$c timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT" -o chunk$c \
    --output-format csv -- python3 $ARGS > "$OUT/chunk$c.log" 2>&1
  echo "== chunk $c"; python3 exp/kstats.py "$OUT"/chunk$c*_kernel_stats.csv
  tail -1 "$OUT/chunk$c.log" | cut -c1-200
done
