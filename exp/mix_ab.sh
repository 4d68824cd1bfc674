#!/bin/bash
# two-stream pairs with one A and one B wave per SIMD (HONK_PAIR_MIX, the default build) vs
# two waves of one role per SIMD (exp/_var/libhonk_nomix.so), alternating: res8 (C3), res15 bf16
set -o pipefail
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/mix
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_res_kernels.py tests/test_gpu_bf16.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for rep in 1 2; do
for v in default nomix; do
  if [ $v = default ]; then unset HONK_LIB; else export HONK_LIB=$PWD/exp/_var/libhonk_$v.so; fi
  for m in res8 res15; do
    timeout -k 10 200 python -u bench.py --model $m --precision bf16 --batch 131072 --steps 8 --warmup 2 --no-alt --no-cpu-baseline > $OUT/b_${m}_$v.json 2> $OUT/b_${m}_$v.err || exit 1
    python -c "import json; d=json.load(open('$OUT/b_${m}_$v.json')); print('$m $v', d['value'], d['roofline'].get('avg_ms_per_layer'), d['parity']['max_abs_logit_err_vs_oracle_f64'])"
  done
done
done
