#!/bin/bash
# rocprofv3 kernel-trace + FETCH_SIZE + WRITE_SIZE passes (each its own run) for the
# bench's secondary configs, so every roofline sub-object carries a PMC traffic:
#   c2f  cnn-trad-pool2 f32      (65,536 clips per step)
#   c2x  cnn-trad-pool2 bf16x3
#   c3   res8 bf16               (8192-clip chunks, two per step)
#   c5   res26-narrow training   (4096 clips, 1 warmup + 1 timed step)
# then on the CPU side:  python tools/pmc_summary.py gpurun_out/prof <tag>_c2f 65536 cnn-trad-pool2  (etc.)
set -e
TAG=${1:-r3}
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/prof
mkdir -p "$OUT"
run3() {  # name, bench args
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT" -o ${TAG}_${n}_trace --output-format csv -- python3 bench.py "$@" > "$OUT/${TAG}_${n}_trace.log" 2>&1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT" -o ${TAG}_${n}_fetch --output-format csv -- python3 bench.py "$@" > "$OUT/${TAG}_${n}_fetch.log" 2>&1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT" -o ${TAG}_${n}_write --output-format csv -- python3 bench.py "$@" > "$OUT/${TAG}_${n}_write.log" 2>&1
  echo "[profile_configs] $n done"
}
run3 c2f --model cnn-trad-pool2 --precision f32 --steps 1 --warmup 1 --no-alt --no-cpu-baseline
run3 c2x --model cnn-trad-pool2 --precision bf16x3 --steps 1 --warmup 1 --no-alt --no-cpu-baseline
run3 c3 --model res8 --precision bf16 --batch 16384 --steps 1 --warmup 1 --no-alt --no-cpu-baseline
HONK_BENCH_TRAIN_PARITY=0 run3 c5 --train --steps 1 --warmup 1
