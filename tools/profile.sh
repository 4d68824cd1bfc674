#!/bin/bash
# rocprofv3 passes for the bench workload (run on the GPU box from the repo root):
#   1. kernel trace + stats (bench defaults) -> gpurun_out/prof/<tag>_trace*
#   2. PMC FETCH_SIZE  (own pass)    -> gpurun_out/prof/<tag>_fetch*
#   3. PMC WRITE_SIZE  (own pass)    -> gpurun_out/prof/<tag>_write*
# The profiled program is python3 itself (no launcher hop after `--`).
set -e
TAG=${1:-r1}
BATCH=${BATCH:-16384}
STEPS=${STEPS:-2}
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/prof
mkdir -p "$OUT"
ARGS="bench.py --batch $BATCH --steps $STEPS --warmup 1 --no-cpu-baseline ${PROF_EXTRA:---no-configs}"
# the trace pass runs the bench's own default workload and steps (131,072 clips per step):
# its kernel averages are taken at the clock the timed bench holds (a short 16K-clip run
# measures the pair kernel ~13 % faster: the chip has not lowered its clock yet)
TARGS="bench.py --no-cpu-baseline ${PROF_EXTRA:---no-configs}"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT" -o ${TAG}_trace --output-format csv -- python3 $TARGS > "$OUT/${TAG}_trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT" -o ${TAG}_fetch --output-format csv -- python3 $ARGS > "$OUT/${TAG}_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT" -o ${TAG}_write --output-format csv -- python3 $ARGS > "$OUT/${TAG}_write.log" 2>&1
find "$OUT" -name "*.csv" | head -50
