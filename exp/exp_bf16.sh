#!/bin/bash
# round 4: bf16 pair (NS = 2) after the partial-spill fix, the device data path, an f16x2 profile
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
T="tests/test_gpu_bf16.py tests/test_gpu_res_kernels.py tests/test_nonfinite.py tests/test_device_data.py tests/test_gpu_f16x2.py"
timeout -k 10 600 python -u -m pytest $T -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/e2_tests.log 2>&1
echo "tests rc=$?"; tail -8 gpurun_out/e2_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o r4c_f16 --output-format csv -- python3 bench.py --precision f16x2 --no-alt --no-cpu-baseline --steps 2 > gpurun_out/prof/r4c_f16.log 2>&1
echo "prof rc=$?"
