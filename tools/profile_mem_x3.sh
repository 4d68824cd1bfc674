#!/bin/bash
# memory-pipeline counter passes (each its own run, --kernel-trace only) for the
# bf16x3 block kernel: TA/TD/TCP busy and stall cycles, then TCC busy/stalls
set -e
TAG=${1:-r1}
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/prof
mkdir -p "$OUT"
ARGS="bench.py --precision bf16x3 --batch 8192 --steps 1 --warmup 0 --no-cpu-baseline --no-alt"
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_LFIFO_STALL_CYCLES_sum GRBM_GUI_ACTIVE --kernel-trace -d "$OUT" -o ${TAG}_x3_tatd --output-format csv -- python3 $ARGS > "$OUT/${TAG}_x3_tatd.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_BUSY_sum TCC_TAG_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum TCC_HIT_sum GRBM_GUI_ACTIVE --kernel-trace -d "$OUT" -o ${TAG}_x3_tcc --output-format csv -- python3 $ARGS > "$OUT/${TAG}_x3_tcc.log" 2>&1
