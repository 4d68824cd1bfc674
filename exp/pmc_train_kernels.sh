#!/bin/bash
# SQ counters of the three C5 training conv kernels (exp/train_kernels_once.py), one pass.
set -e
export TMPDIR=/tmp
TAG=${1:-tk}
OUT=$PWD/gpurun_out/prof
mkdir -p "$OUT"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace -d "$OUT" -o ${TAG}_sq --output-format csv -- python3 exp/train_kernels_once.py > "$OUT/${TAG}_sq.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE --kernel-trace -d "$OUT" -o ${TAG}_sq2 --output-format csv -- python3 exp/train_kernels_once.py > "$OUT/${TAG}_sq2.log" 2>&1
PMC_FILTER=train:: python3 exp/pmc_print.py "$OUT"/${TAG}_sq_counter_collection.csv "$OUT"/${TAG}_sq2_counter_collection.csv
