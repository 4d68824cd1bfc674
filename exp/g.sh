mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 300 python exp/pair_exp.py time prev base prev base > gpurun_out/pair_r5z.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5w_pytest.log 2>&1
