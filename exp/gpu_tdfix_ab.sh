# C5 A/B: conv3x3d_kernel with the compile-time res26-narrow geometry (default) vs runtime (HONK_TD_FIXED=0)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  HONK_TD_FIXED=0 timeout -k 10 200 python -u bench.py --train --steps 10 --warmup 2 > gpurun_out/tdf_off_$i.json 2>/dev/null
  timeout -k 10 200 python -u bench.py --train --steps 10 --warmup 2 > gpurun_out/tdf_on_$i.json 2>/dev/null
  grep -o '"value": [0-9.]*' gpurun_out/tdf_off_$i.json gpurun_out/tdf_on_$i.json
done
timeout -k 10 600 python -u -m pytest -m gpu tests/test_gpu_train_native.py tests/test_train_golden.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tdf_pytest.log 2>&1
tail -2 gpurun_out/tdf_pytest.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o tdf_trace --output-format csv -- python3 bench.py --train --steps 2 --warmup 1 > gpurun_out/tdf_prof.log 2>&1
