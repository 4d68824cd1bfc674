# C5 A/B: the in-tree build without / with the fused tails
# (HONK_TRAIN_FUSE_TAIL=0 / 1), alternating; then the training GPU tests and a trace
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do

  HONK_TRAIN_FUSE_TAIL=0 timeout -k 10 200 python -u bench.py --train --steps 10 --warmup 2 > gpurun_out/tab_nofuse_$i.json 2>/dev/null
  timeout -k 10 200 python -u bench.py --train --steps 10 --warmup 2 > gpurun_out/tab_new_$i.json 2>/dev/null
  grep -o '"value": [0-9.]*' gpurun_out/tab_nofuse_$i.json gpurun_out/tab_new_$i.json
done
timeout -k 10 600 python -u -m pytest -m gpu tests/test_gpu_train_native.py tests/test_train_golden.py tests/test_gpu_cnn_train.py tests/test_gpu_head.py tests/test_gpu_train_envelope.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tab_pytest.log 2>&1
tail -2 gpurun_out/tab_pytest.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o tab_trace --output-format csv -- python3 bench.py --train --steps 2 --warmup 1 > gpurun_out/tab_prof.log 2>&1
