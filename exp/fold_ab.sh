#!/bin/bash
# C5: the folded BatchNorm's in-LDS rewrite of the next tile done by each wave after its super
# tiles (default build) vs at the top of the tile between the DMA wait and the barrier
# (exp/_var/libhonk_oldfold.so, exp/build_variant.sh ... train), alternating on one box
set -o pipefail
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/fold
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_train_native.py tests/test_train_golden.py tests/test_syncbn.py -m gpu > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for rep in 1 2; do
for v in default oldfold; do
  if [ $v = default ]; then unset HONK_LIB; else export HONK_LIB=$PWD/exp/_var/libhonk_$v.so; fi
  HONK_BENCH_TRAIN_PARITY=0 timeout -k 10 300 python -u bench.py --train --steps 4 --warmup 1 --no-alt --no-cpu-baseline > $OUT/c5_$v.json 2> $OUT/c5_$v.err || exit 1
  python -c "import json; d=json.load(open('$OUT/c5_$v.json')); print('c5 $v', d['value'])"
done
done
unset HONK_LIB
HONK_BENCH_TRAIN_PARITY=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT -o tr --output-format csv -- python3 bench.py --train --steps 1 --warmup 1 --no-alt --no-cpu-baseline > $OUT/tr.log 2>&1 || exit 1
python - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/fold/**/tr_kernel_stats.csv',recursive=True)[0]
for r in sorted(csv.DictReader(open(f)),key=lambda r:-float(r['TotalDurationNs']))[:5]:
    print(f"{float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>4} {r['Name'][:90]}")
PY
