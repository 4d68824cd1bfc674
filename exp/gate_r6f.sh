#!/bin/bash
# GPU tests after the pooled-map chunk change, then the secondary configs' profiles
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6f_pytest.log 2>&1 || { tail -30 gpurun_out/r6f_pytest.log; exit 1; }
tail -1 gpurun_out/r6f_pytest.log
tools/profile_configs.sh r6f
