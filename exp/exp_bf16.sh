#!/bin/bash
# round 4: bf16 pair (NS = 2) after the partial-spill fix, MFMA conv0, the device data
# path, f16x2; an f16x2 kernel profile; C3 (res8 bf16) with the MFMA / VALU conv0 and pairs
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
T="tests/test_gpu_bf16.py tests/test_gpu_res_kernels.py tests/test_nonfinite.py tests/test_device_data.py tests/test_gpu_f16x2.py tests/test_gpu_bf16x3.py"
timeout -k 10 600 python -u -m pytest $T -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/e2_tests.log 2>&1
echo "tests rc=$?"; tail -8 gpurun_out/e2_tests.log
C3="--model res8 --precision bf16 --batch 131072 --no-alt --no-cpu-baseline --steps 5"
timeout -k 10 200 python -u bench.py $C3 > gpurun_out/e2_c3.json 2>/dev/null; echo "c3 rc=$?"
HONK_CONV0=v timeout -k 10 200 python -u bench.py $C3 > gpurun_out/e2_c3_valu.json 2>/dev/null; echo "c3v rc=$?"
HONK_RES_KERNEL=w timeout -k 10 200 python -u bench.py $C3 > gpurun_out/e2_c3_w.json 2>/dev/null; echo "c3w rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o r4c_f16 --output-format csv -- python3 bench.py --precision f16x2 --no-alt --no-cpu-baseline --steps 2 > gpurun_out/prof/r4c_f16.log 2>&1
echo "prof rc=$?"
