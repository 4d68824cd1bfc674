#!/bin/bash
# the res GPU tests touched by the C3 path, then C3 / res26 bf16 / res15 bf16 benches
set -o pipefail
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/c3g
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread tests/test_gpu_res_kernels.py tests/test_gpu_bf16.py tests/test_nonfinite.py tests/test_gpu_parity.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
grep -E "pairs max|conv0p vs" $OUT/tests.log | head
for m in res8 res26 res15; do
  timeout -k 10 200 python -u bench.py --model $m --precision bf16 --batch 131072 --steps 10 --warmup 2 --no-alt --no-cpu-baseline > $OUT/b_${m}.json 2> $OUT/b_${m}.err || exit 1
  python -c "import json; d=json.load(open('$OUT/b_${m}.json')); print('$m', d['value'], d['parity'])"
done
