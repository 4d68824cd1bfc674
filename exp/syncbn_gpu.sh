#!/bin/bash
# SyncBN on the GPU (2 gloo ranks on cuda:0) + the training GPU tests it touches
set -o pipefail
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/sbn
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_syncbn.py tests/test_train_golden.py tests/test_gpu_train_native.py -m gpu > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
