#!/bin/bash
# SQ counters of the headline (res15 f16x2) kernels: one pass (8 SQ counters + GRBM)
set -e
TAG=${1:-r4}
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/prof
mkdir -p "$OUT"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace -d "$OUT" -o ${TAG}_pairsq --output-format csv -- python3 bench.py --batch 16384 --steps 1 --warmup 1 --no-cpu-baseline --no-alt > "$OUT/${TAG}_pairsq.log" 2>&1
echo "[profile_sq_pair] done"
