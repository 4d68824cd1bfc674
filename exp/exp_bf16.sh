#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
T="tests/test_gpu_bf16.py tests/test_gpu_res_kernels.py"
HONK_PAIR_STREAMS=1 timeout -k 10 300 python -u -m pytest $T -m gpu -q -k bf16 --timeout 120 --timeout-method thread > gpurun_out/e1_streams1.log 2>&1
echo "streams1 rc=$?"; tail -3 gpurun_out/e1_streams1.log
HONK_LIB=$PWD/exp/_var/libhonk_intmax.so timeout -k 10 300 python -u -m pytest $T -m gpu -q -k bf16 --timeout 120 --timeout-method thread > gpurun_out/e1_intmax.log 2>&1
echo "intmax rc=$?"; tail -3 gpurun_out/e1_intmax.log
timeout -k 10 300 python -u -m pytest tests/test_device_data.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/e1_data.log 2>&1
echo "data rc=$?"; tail -3 gpurun_out/e1_data.log
