#!/bin/bash
# SQ/GRBM + FETCH passes for the bf16 block kernel
set -e
TAG=${1:-r1}
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/prof
mkdir -p "$OUT"
ARGS="bench.py --precision bf16 --batch 8192 --steps 1 --warmup 0 --no-cpu-baseline --no-alt"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT" -o ${TAG}_b16trace --output-format csv -- python3 $ARGS > "$OUT/${TAG}_b16trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace -d "$OUT" -o ${TAG}_b16sq --output-format csv -- python3 $ARGS > "$OUT/${TAG}_b16sq.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT" -o ${TAG}_b16fetch --output-format csv -- python3 $ARGS > "$OUT/${TAG}_b16fetch.log" 2>&1
