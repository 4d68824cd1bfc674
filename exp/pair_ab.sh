#!/bin/bash
# Same-box A/B of pair-kernel variants (exp/build_vf_variant.sh builds them into exp/_var):
# the default build vs each HONK_LIB variant, alternating, res15 f16x2 bench
set -o pipefail
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/pab
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_f16x2.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for rep in 1 2; do
for v in default "$@"; do
  if [ $v = default ]; then unset HONK_LIB; else export HONK_LIB=$PWD/exp/_var/libhonk_$v.so; fi
  timeout -k 10 200 python -u bench.py --no-alt --no-cpu-baseline --steps 10 --warmup 2 > $OUT/b_$v.json 2> $OUT/b_$v.err || exit 1
  python -c "import json; d=json.load(open('$OUT/b_$v.json')); print('$v', d['value'], d['roofline'].get('avg_ms_per_layer'), d['parity']['max_abs_logit_err_vs_oracle_f64'])"
done
done
