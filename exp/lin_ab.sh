#!/bin/bash
# linear A-in DMA (block16p_body LIN, the default on res8 / res26 bf16) vs the row pieces
# (HONK_PAIR_LIN=0), alternating on one box; GPU tests of the res paths first
set -o pipefail
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/lin
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread tests/test_gpu_res_kernels.py tests/test_gpu_bf16.py tests/test_nonfinite.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
grep -E "pairs max" $OUT/tests.log | head
for m in res8 res26; do
for v in d 0 d 0; do
  if [ $v = 0 ]; then export HONK_PAIR_LIN=0; else unset HONK_PAIR_LIN; fi
  timeout -k 10 200 python -u bench.py --model $m --precision bf16 --batch 131072 --steps 10 --warmup 2 --no-alt --no-cpu-baseline > $OUT/b_${m}_$v.json 2> $OUT/b_${m}_$v.err || exit 1
  python -c "import json; d=json.load(open('$OUT/b_${m}_$v.json')); print('$m $v', d['value'], d['roofline'].get('avg_ms_per_layer'), d['parity'])"
done
done
unset HONK_PAIR_LIN
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT -o tr --output-format csv -- python3 bench.py --model res8 --precision bf16 --batch 131072 --steps 2 --warmup 1 --no-alt --no-cpu-baseline > $OUT/tr.log 2>&1 || exit 1
python - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/lin/**/tr_kernel_stats.csv',recursive=True)[0]
for r in sorted(csv.DictReader(open(f)),key=lambda r:-float(r['TotalDurationNs']))[:5]:
    print(f"{float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>4} {r['Name'][:100]}")
PY
