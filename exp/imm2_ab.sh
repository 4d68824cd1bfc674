#!/bin/bash
# bf16 two-stream tap-step pairs (default) vs the row-table pairs (HONK_PAIR_IMM2=0), res15
set -o pipefail
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/imm2
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_res_kernels.py tests/test_gpu_bf16.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in d 0 d 0; do
  if [ $v = 0 ]; then export HONK_PAIR_IMM2=0; else unset HONK_PAIR_IMM2; fi
  timeout -k 10 200 python -u bench.py --precision bf16 --steps 8 --warmup 2 --no-alt --no-cpu-baseline > $OUT/b_$v.json 2> $OUT/b_$v.err || exit 1
  python -c "import json; d=json.load(open('$OUT/b_$v.json')); print('res15 bf16 $v', d['value'], d['roofline'].get('avg_ms_per_layer'), d['parity'])"
done
unset HONK_PAIR_IMM2
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT -o tr --output-format csv -- python3 bench.py --precision bf16 --steps 2 --warmup 1 --no-alt --no-cpu-baseline > $OUT/tr.log 2>&1 || exit 1
python - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/imm2/**/tr_kernel_stats.csv',recursive=True)[0]
for r in sorted(csv.DictReader(open(f)),key=lambda r:-float(r['TotalDurationNs']))[:8]:
    print(f"{float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>4} {r['Name'][:100]}")
PY
