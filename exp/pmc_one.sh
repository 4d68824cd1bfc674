#!/bin/bash
# One PMC pass (MFMA busy, clock) of the res15 bf16x3 forward with an optional HONK_LIB.
set -e
export TMPDIR=/tmp
TAG=${1:-one}
OUT=$PWD/gpurun_out/prof
mkdir -p "$OUT"
ARGS="bench.py --batch 8192 --steps 1 --warmup 0 --no-cpu-baseline --no-alt --no-configs"
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE --kernel-trace -d "$OUT" -o ${TAG} --output-format csv -- python3 $ARGS > "$OUT/${TAG}.log" 2>&1
python3 exp/pmc_print.py "$OUT"/${TAG}_counter_collection.csv
python3 - "$OUT"/${TAG}_kernel_trace.csv <<'PY'
import csv, sys, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if "block16" in n:
        d[n.split("(")[0][-40:]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for k, v in d.items():
    print(k, "mean ms", sum(v) / len(v), "n", len(v))
PY
