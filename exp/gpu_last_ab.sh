set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_res_kernels.py tests/test_gpu_bf16x3.py tests/test_gpu_bf16.py tests/test_gpu_train_native.py -x -q --timeout 120 --timeout-method thread > gpurun_out/g1_pytest.log 2>&1
tail -2 gpurun_out/g1_pytest.log
timeout -k 10 300 python -u bench.py --no-configs --no-cpu-baseline > gpurun_out/g1_bench_l.json 2> gpurun_out/g1_bench_l.err
HONK_LAST_KERNEL=w timeout -k 10 300 python -u bench.py --no-configs --no-cpu-baseline > gpurun_out/g1_bench_w.json 2> gpurun_out/g1_bench_w.err
HONK_LAST_NS=2 timeout -k 10 300 python -u bench.py --precision bf16 --no-alt --no-cpu-baseline > gpurun_out/g1_bench_ns2.json 2> gpurun_out/g1_bench_ns2.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o g1_trace --output-format csv -- python3 bench.py --batch 16384 --steps 2 --warmup 1 --no-cpu-baseline --no-configs > gpurun_out/g1_prof.log 2>&1
echo done
