set -e
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/prof
mkdir -p "$OUT"
for v in 1 0; do
HONK_PAIR_KS=$v timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace -d "$OUT" -o ks${v}_pairsq --output-format csv -- python3 bench.py --batch 16384 --steps 1 --warmup 1 --no-cpu-baseline --no-alt > "$OUT/ks${v}_pairsq.log" 2>&1
done
for v in 1 0; do
HONK_PAIR_KS=$v timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace -d "$OUT" -o ks${v}_pairsq2 --output-format csv -- python3 bench.py --batch 16384 --steps 1 --warmup 1 --no-cpu-baseline --no-alt > "$OUT/ks${v}_pairsq2.log" 2>&1
done
ls $OUT
