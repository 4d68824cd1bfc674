#!/bin/bash
# Chunk size (HONK_RES_CHUNK: clips per forward launch sequence) on res8 bf16 (C3) and res15
# bf16 / f16x2, alternating on one box
set -o pipefail
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/chunk
mkdir -p $OUT
for rep in 1 2; do
for c in 4096 8192 16384 32768; do
  HONK_RES_CHUNK=$c timeout -k 10 200 python -u bench.py --model res8 --precision bf16 --batch 131072 --steps 10 --warmup 2 --no-alt --no-cpu-baseline > $OUT/b_res8_$c.json 2> $OUT/b_res8_$c.err || exit 1
  python -c "import json; d=json.load(open('$OUT/b_res8_$c.json')); print('res8 bf16 chunk $c', d['value'], d['parity'])"
done
done
for rep in 1 2; do
for p in bf16 f16x2; do
for c in 4096 8192; do
  HONK_RES_CHUNK=$c timeout -k 10 200 python -u bench.py --precision $p --steps 8 --warmup 2 --no-alt --no-cpu-baseline > $OUT/b_res15_${p}_$c.json 2> $OUT/b_res15_${p}_$c.err || exit 1
  python -c "import json; d=json.load(open('$OUT/b_res15_${p}_$c.json')); print('res15 $p chunk $c', d['value'])"
done
done
done
