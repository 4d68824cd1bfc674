#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
C3="bench.py --model res8 --precision bf16 --batch 16384 --no-alt --no-cpu-baseline --steps 1 --warmup 1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace -d gpurun_out/prof -o r4d_c3sq --output-format csv -- python3 $C3 > gpurun_out/prof/r4d_c3sq.log 2>&1
echo "sq rc=$?"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/prof -o r4d_c3sq2 --output-format csv -- python3 $C3 > gpurun_out/prof/r4d_c3sq2.log 2>&1
echo "sq2 rc=$?"
