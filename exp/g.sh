mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 300 python exp/pair_exp.py time f16tu vf f16tu vf > gpurun_out/pair_r5vf.log 2>&1 && \
PAIR_PREC=bf16x3 timeout -k 10 300 python exp/pair_exp.py time f16tu vf f16tu vf >> gpurun_out/pair_r5vf.log 2>&1 && \
PAIR_PREC=bf16 timeout -k 10 300 python exp/pair_exp.py time f16tu vf f16tu vf >> gpurun_out/pair_r5vf.log 2>&1
