#!/bin/bash
# PMC passes for the bf16x3 row-band kernel (res15): one counter group per run
# (<= 8 SQ, <= 2 TA, 1 GRBM per pass), kernel-trace only, each pass under its own
# hard time limit.  Summaries land in gpurun_out/prof/<tag>_g<i>_counter_collection.csv.
set -e
TAG=${1:-rb}
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/prof
mkdir -p "$OUT"
ARGS="bench.py --precision bf16x3 --batch 8192 --steps 1 --warmup 0 --no-cpu-baseline --no-alt"
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INSTS_VMEM GRBM_GUI_ACTIVE" \
           "TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -d "$OUT" -o ${TAG}_g$i --output-format csv -- python3 $ARGS > "$OUT/${TAG}_g$i.log" 2>&1
done
