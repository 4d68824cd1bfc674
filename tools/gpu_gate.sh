#!/bin/bash
# Round-end style gate on the GPU box: GPU parity tests, smoke(), default bench, rocprof stats.
# Every GPU step has its own time limit; steps are chained so a failure stops the script.
set -e
TAG=${1:-r1h}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
tools/profile.sh ${TAG}
