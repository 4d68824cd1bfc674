set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
HONK_TRAIN_FOLD_BN=1 HONK_BENCH_TRAIN_PARITY=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/foldprof -o on --output-format csv -- python3 bench.py --train --steps 2 --warmup 1 > gpurun_out/fold_prof_on.log 2>&1 && \
HONK_TRAIN_FOLD_BN=0 HONK_BENCH_TRAIN_PARITY=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/foldprof -o off --output-format csv -- python3 bench.py --train --steps 2 --warmup 1 > gpurun_out/fold_prof_off.log 2>&1
rc=$?
find gpurun_out/foldprof -name "*kernel_stats.csv" | sort
exit $rc
