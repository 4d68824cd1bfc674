#!/bin/bash
# SQ counter passes on the res15 bf16x3 forward (fused pair + weight-stationary kernels),
# one counter group per run, each under its own hard limit.
set -e
export TMPDIR=/tmp
TAG=${1:-pp}
OUT=$PWD/gpurun_out/prof
mkdir -p "$OUT"
ARGS="bench.py --batch 8192 --steps 1 --warmup 0 --no-cpu-baseline --no-alt --no-configs"
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -d "$OUT" -o ${TAG}_g$i --output-format csv -- python3 $ARGS > "$OUT/${TAG}_g$i.log" 2>&1
done
python3 exp/pmc_print.py "$OUT"/${TAG}_g*_counter_collection.csv
