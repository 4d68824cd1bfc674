#!/bin/bash
# Closing gate + every PMC pass the bench's roofline objects read:
#   tools/gpu_gate.sh TAG        (GPU tests, smoke, bench, --gpus 2 rehearsal, res15 trace/FETCH/WRITE)
#   tools/profile_configs.sh TAG (C2 f32 / bf16x3, C3, C5: trace/FETCH/WRITE)
#   one SQ pass over the C5 training step
set -e
TAG=${1:-r3}
export TMPDIR=/tmp
tools/gpu_gate.sh $TAG
tools/profile_configs.sh $TAG
OUT=$PWD/gpurun_out/prof
HONK_BENCH_TRAIN_PARITY=0 timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace -d "$OUT" -o ${TAG}_c5sq --output-format csv -- python3 bench.py --train --steps 1 --warmup 1 > "$OUT/${TAG}_c5sq.log" 2>&1
echo "[gate_full] done"
