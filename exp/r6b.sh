set -o pipefail
export TMPDIR=/tmp
HONK_PAIR_STREAMS=3 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bf16.py tests/test_gpu_res_kernels.py > gpurun_out/r6c_tests.log 2>&1 || { tail -30 gpurun_out/r6c_tests.log; exit 1; }
tail -2 gpurun_out/r6c_tests.log
grep -E "x 1024|tie" gpurun_out/r6c_tests.log | head
for v in 3 1 3 1; do
HONK_PAIR_STREAMS=$v timeout -k 10 200 python -u bench.py --precision bf16 --no-alt --no-cpu-baseline --steps 10 > gpurun_out/r6c_bench_$v.json 2> gpurun_out/r6c_bench_$v.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/r6c_bench_$v.json')); print('streams $v', d['value'], d['roofline'].get('avg_ms_per_layer'), d['parity'])"
done
