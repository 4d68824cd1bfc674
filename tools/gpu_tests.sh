#!/bin/bash
# GPU test pass: the named test files first (exit 0/1 = ran), then the whole -m gpu suite.
# A fault, abort, segfault or time limit (any other status) stops the script there.
TAG=${1:-r3}
shift
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_first.log 2>&1
  rc=$?
  tail -5 gpurun_out/${TAG}_first.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
tail -5 gpurun_out/${TAG}_pytest.log
exit $rc
