#!/bin/bash
# SQ counters of C3's kernels (res8 bf16: the pair, conv0p, tail_act), two passes
set -e
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/c3sq
mkdir -p "$OUT"
A="bench.py --model res8 --precision bf16 --batch 16384 --steps 1 --warmup 1 --no-cpu-baseline --no-alt"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace -d "$OUT" -o sq1 --output-format csv -- python3 $A > "$OUT/sq1.log" 2>&1
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAVES SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-trace -d "$OUT" -o sq2 --output-format csv -- python3 $A > "$OUT/sq2.log" 2>&1
ls "$OUT"
