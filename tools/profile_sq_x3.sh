#!/bin/bash
# SQ/GRBM counter pass (own run, --kernel-trace only) for the bf16x3 block kernel:
# MFMA busy, LDS array activity / bank conflicts, wait breakdown.
set -e
TAG=${1:-r1}
PREC=${PREC:-bf16x3}
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/prof
mkdir -p "$OUT"
ARGS="bench.py --precision $PREC --batch 8192 --steps 1 --warmup 0 --no-cpu-baseline --no-alt"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace -d "$OUT" -o ${TAG}_${PREC}_sq --output-format csv -- python3 $ARGS > "$OUT/${TAG}_${PREC}_sq.log" 2>&1
