#!/bin/bash
# SQ/GRBM counter pass for the dominant kernel (own rocprofv3 pass, kernel trace only).
set -e
TAG=${1:-r1}
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/prof
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace -d "$OUT" -o ${TAG}_sq --output-format csv -- python3 bench.py --batch 8192 --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/${TAG}_sq.log" 2>&1
