#!/bin/bash
# bf16: the res/bf16 GPU tests (single-stream tap-step pairs, last layer), then res15 bf16
# with the row-table tap-step last layer (default) vs HONK_LAST_KERNEL=w-free baseline:
# the bench twice and a kernel trace
set -o pipefail
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/bfl
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_res_kernels.py tests/test_gpu_bf16.py tests/test_nonfinite.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in 1 2; do
  timeout -k 10 200 python -u bench.py --precision bf16 --steps 8 --warmup 2 --no-alt --no-cpu-baseline > $OUT/b_$v.json 2> $OUT/b_$v.err || exit 1
  python -c "import json; d=json.load(open('$OUT/b_$v.json')); print('res15 bf16', d['value'], d['parity'])"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT -o tr --output-format csv -- python3 bench.py --precision bf16 --steps 2 --warmup 1 --no-alt --no-cpu-baseline > $OUT/tr.log 2>&1 || exit 1
python - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/bfl/**/tr_kernel_stats.csv',recursive=True)[0]
for r in sorted(csv.DictReader(open(f)),key=lambda r:-float(r['TotalDurationNs']))[:5]:
    print(f"{float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>4} {r['Name'][:100]}")
PY
