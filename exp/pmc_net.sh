#!/bin/bash
# Kernel times + SQ counters of the res8 bf16 forward (C3) on the whole-stack kernel.
set -e
export TMPDIR=/tmp
TAG=${1:-net}
OUT=$PWD/gpurun_out/prof
mkdir -p "$OUT"
ARGS="bench.py --model res8 --precision bf16 --batch 16384 --steps 1 --warmup 1 --no-alt --no-cpu-baseline"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT" -o ${TAG}_trace --output-format csv -- python3 $ARGS > "$OUT/${TAG}_trace.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace -d "$OUT" -o ${TAG}_sq --output-format csv -- python3 $ARGS > "$OUT/${TAG}_sq.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE --kernel-trace -d "$OUT" -o ${TAG}_sq2 --output-format csv -- python3 $ARGS > "$OUT/${TAG}_sq2.log" 2>&1
python3 - "$OUT"/${TAG}_trace_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "res::" in r["Name"]:
        print(f'{r["Name"][:70]:70s} calls {r["Calls"]:>5s} avg {float(r["AverageNs"])/1e3:9.1f} us')
PY
PMC_FILTER=res:: python3 exp/pmc_print.py "$OUT"/${TAG}_sq_counter_collection.csv "$OUT"/${TAG}_sq2_counter_collection.csv
