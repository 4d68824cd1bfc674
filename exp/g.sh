mkdir -p gpurun_out && export TMPDIR=/tmp && \
PAIR_PREC=bf16 timeout -k 10 400 python exp/pair_exp.py time vf pin26 pin28 vf pin26 pin28 > gpurun_out/pin_ab2.log 2>&1
