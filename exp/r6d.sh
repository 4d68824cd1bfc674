set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_f16x2.py -k "ksplit or launch_plan or golden or invariance or large" > gpurun_out/r6d_tests.log 2>&1 || { tail -40 gpurun_out/r6d_tests.log; exit 1; }; tail -1 gpurun_out/r6d_tests.log
grep -E "FAIL|k-split" gpurun_out/r6d_tests.log | tail -20
for v in 1 0 1 0; do
HONK_PAIR_KS=$v timeout -k 10 200 python -u bench.py --no-alt --no-cpu-baseline --steps 10 > gpurun_out/r6d_bench_$v.json 2> gpurun_out/r6d_bench_$v.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/r6d_bench_$v.json')); print('ks $v', d['value'], d['roofline'].get('avg_ms_per_layer'), d['parity'])"
done
