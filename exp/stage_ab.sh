#!/bin/bash
# conv0m / conv0p staging with every load of a thread in flight (default build) vs the
# previous one-load-at-a-time loop (exp/_var/libhonk_oldstage.so, exp/build_variant.sh),
# alternating on one box: C3 (res8 bf16) and res15 f16x2
set -o pipefail
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/stage
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_res_kernels.py tests/test_gpu_bf16.py tests/test_gpu_f16x2.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for rep in 1 2; do
for v in default oldstage; do
  if [ $v = default ]; then unset HONK_LIB; else export HONK_LIB=$PWD/exp/_var/libhonk_$v.so; fi
  timeout -k 10 200 python -u bench.py --model res8 --precision bf16 --batch 131072 --steps 10 --warmup 2 --no-alt --no-cpu-baseline > $OUT/c3_$v.json 2> $OUT/c3_$v.err || exit 1
  python -c "import json; d=json.load(open('$OUT/c3_$v.json')); print('c3 $v', d['value'])"
  timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 --no-alt --no-cpu-baseline > $OUT/h_$v.json 2> $OUT/h_$v.err || exit 1
  python -c "import json; d=json.load(open('$OUT/h_$v.json')); print('res15 $v', d['value'])"
done
done
unset HONK_LIB
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT -o tr --output-format csv -- python3 bench.py --model res8 --precision bf16 --batch 16384 --steps 2 --warmup 1 --no-alt --no-cpu-baseline > $OUT/tr.log 2>&1 || exit 1
python - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/stage/**/tr_kernel_stats.csv',recursive=True)[0]
for r in sorted(csv.DictReader(open(f)),key=lambda r:-float(r['TotalDurationNs']))[:4]:
    print(f"{float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>4} {r['Name'][:90]}")
PY
