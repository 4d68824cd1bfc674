set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
L="exp/_var/libhonk_nag64.so exp/_var/libhonk_nag28.so exp/_var/libhonk_nag32.so exp/_var/libhonk_nag24.so"
PREC=bf16 timeout -k 10 400 python -u exp/lib_ab.py $L > gpurun_out/nag_bf16.log 2>&1
cat gpurun_out/nag_bf16.log
