#!/bin/bash
# C3 (res8 bf16): the default (round 6: three fused pairs on the two-stream kernel +
# act_chsum_kernel) against HONK_RES_KERNEL=r (round 5's row-band layers), alternating on
# one box; res26 bf16 likewise; then a kernel trace of each res8 path
set -o pipefail
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/c3ab
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_res_kernels.py tests/test_gpu_bf16.py tests/test_gpu_parity.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
grep -E "pairs max|tie|x 1024" $OUT/tests.log | head
for m in res8 res26; do
for v in d r d r; do
  if [ $v = r ]; then export HONK_RES_KERNEL=r; else unset HONK_RES_KERNEL; fi
  timeout -k 10 200 python -u bench.py --model $m --precision bf16 --batch 131072 --steps 10 --warmup 2 --no-alt --no-cpu-baseline > $OUT/b_${m}_$v.json 2> $OUT/b_${m}_$v.err || exit 1
  python -c "import json; d=json.load(open('$OUT/b_${m}_$v.json')); print('$m $v', d['value'], d['roofline'].get('avg_ms_per_layer'), d['parity'])"
done
done
for v in d r; do
  if [ $v = r ]; then export HONK_RES_KERNEL=r; else unset HONK_RES_KERNEL; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT -o tr_$v --output-format csv -- python3 bench.py --model res8 --precision bf16 --batch 16384 --steps 2 --warmup 1 --no-alt --no-cpu-baseline > $OUT/tr_$v.log 2>&1 || exit 1
done
python - <<'PY'
import csv,glob
for v in 'dr':
    f=glob.glob(f'gpurun_out/c3ab/**/tr_{v}_kernel_stats.csv',recursive=True)[0]
    for r in sorted(csv.DictReader(open(f)),key=lambda r:-float(r['TotalDurationNs']))[:7]:
        print(v, f"{float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>4} {r['Name'][:90]}")
PY
