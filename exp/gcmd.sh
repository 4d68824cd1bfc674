mkdir -p gpurun_out && cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5f_pytest.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r5f_bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5f_prof -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/r5f_prof.log 2>&1
