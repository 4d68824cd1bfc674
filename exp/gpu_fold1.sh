set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_train_native.py > gpurun_out/fold_tests.log 2>&1 && \
HONK_TRAIN_FOLD_BN=1 timeout -k 10 300 python3 bench.py --train --steps 10 --warmup 3 > gpurun_out/fold_c5.log 2>&1 && \
HONK_TRAIN_FOLD_BN=0 timeout -k 10 300 python3 bench.py --train --steps 10 --warmup 3 > gpurun_out/fold_c5_off.log 2>&1
rc=$?; tail -3 gpurun_out/fold_tests.log; tail -1 gpurun_out/fold_c5.log | cut -c1-400; tail -1 gpurun_out/fold_c5_off.log | cut -c1-400; exit $rc
