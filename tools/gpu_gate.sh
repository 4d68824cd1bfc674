#!/bin/bash
# Round-end style gate on the GPU box: GPU parity tests, smoke(), default bench,
# a 2-rank bench rehearsal on the one GPU (gloo), rocprof stats.
# Every GPU step has its own time limit; steps are chained so a failure stops the script.
set -e
TAG=${1:-r2a}
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "[gate] pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
tail -2 gpurun_out/${TAG}_pytest.log
echo "[gate] smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
echo "[gate] bench"
timeout -k 10 500 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
echo "[gate] bench --gpus 2 rehearsal (gloo, one GPU)"
HONK_BENCH_ONE_GPU=1 HONK_BENCH_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 2 --steps 2 --cpu-seconds 3 > gpurun_out/${TAG}_bench2.json 2> gpurun_out/${TAG}_bench2.err
if [ -z "$NOPROF" ]; then tools/profile.sh ${TAG}; fi
