#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
T="tests/test_gpu_bf16.py tests/test_gpu_res_kernels.py tests/test_nonfinite.py tests/test_gpu_f16x2.py tests/test_gpu_bf16x3.py tests/test_gpu_parity.py"
timeout -k 10 600 python -u -m pytest $T -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/e3_tests.log 2>&1
echo "tests rc=$?"; tail -3 gpurun_out/e3_tests.log
C3="bench.py --model res8 --precision bf16 --batch 131072 --no-alt --no-cpu-baseline --steps 5"
timeout -k 10 200 python -u $C3 > gpurun_out/e3_c3.json 2>/dev/null; echo "c3 rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o r4f_c3 --output-format csv -- python3 bench.py --model res8 --precision bf16 --batch 16384 --no-alt --no-cpu-baseline --steps 2 > gpurun_out/prof/r4f_c3.log 2>&1
echo "prof rc=$?"
