#!/bin/bash
# A/B timing of the res15 bf16x3 forward: fused pairs (default) vs weight-stationary only.
set -e
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/pairab
mkdir -p "$OUT"
ARGS="bench.py --batch 16384 --steps 2 --warmup 1 --no-cpu-baseline --no-configs --no-alt"
for v in ${VARIANTS:-p w p w}; do
  HONK_RES_KERNEL=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT" -o $v \
    --output-format csv -- python3 $ARGS > "$OUT/$v.log" 2>&1
  echo "== $v"; python3 exp/kstats.py "$OUT"/${v}_kernel_stats.csv
  grep -o '"value": [0-9.]*' "$OUT/$v.log" | head -1
done
