#!/bin/bash
# conv0p_kernel (pooled bf16 conv0: shared K layout, one patch per m-tile) vs conv0m_kernel
# (HONK_CONV0=m), alternating on one box: C3 and res26 bf16; then a kernel trace of each
set -o pipefail
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/c0p
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread tests/test_gpu_res_kernels.py -k "conv0 or res8_bf16 or rowband" tests/test_gpu_bf16.py tests/test_nonfinite.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
grep -E "conv0p vs|pairs max|bf16 max" $OUT/tests.log | head -20
for m in res8 res26; do
for v in d m d m; do
  if [ $v = m ]; then export HONK_CONV0=m; else unset HONK_CONV0; fi
  timeout -k 10 200 python -u bench.py --model $m --precision bf16 --batch 131072 --steps 10 --warmup 2 --no-alt --no-cpu-baseline > $OUT/b_${m}_$v.json 2> $OUT/b_${m}_$v.err || exit 1
  python -c "import json; d=json.load(open('$OUT/b_${m}_$v.json')); print('$m $v', d['value'], d['parity'])"
done
done
for v in d m; do
  if [ $v = m ]; then export HONK_CONV0=m; else unset HONK_CONV0; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT -o tr_$v --output-format csv -- python3 bench.py --model res8 --precision bf16 --batch 131072 --steps 2 --warmup 1 --no-alt --no-cpu-baseline > $OUT/tr_$v.log 2>&1 || exit 1
done
python - <<'PY'
import csv,glob
for v in 'dm':
    f=glob.glob(f'gpurun_out/c0p/**/tr_{v}_kernel_stats.csv',recursive=True)[0]
    for r in sorted(csv.DictReader(open(f)),key=lambda r:-float(r['TotalDurationNs']))[:5]:
        print(v, f"{float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>4} {r['Name'][:90]}")
PY
