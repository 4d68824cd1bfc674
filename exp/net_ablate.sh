#!/bin/bash
# Timing-only ablations of block16n_kernel: variant libraries built with -DHONK_NET_ABL=bits
# (1 epilogue, 2 weight copy, 4 DMA, 8 barriers, 16 MFMAs; exp/build_variant.sh), each
# timed by the bench on res8 bf16 (kernel ms per 4096-clip launch, clips/s).
#   build here:  for v in ...; do HONK_VFLAGS=-DHONK_NET_ABL=$v exp/build_variant.sh abl$v honk_amd/csrc; done
export TMPDIR=/tmp
for v in ${VARIANTS:-0 1 2 4 8 16 31}; do
  LIB=$PWD/exp/_var/libhonk_abl$v.so
  r=$(HONK_RES_KERNEL=n HONK_LIB=$LIB timeout -k 10 120 python3 bench.py --model res8 --precision bf16 --batch 32768 --steps 3 --warmup 1 --no-alt --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(round(r['avg_ms_per_layer']*6, 4), d['value'])")
  echo "abl=$v ms_per_launch clips/s: $r"
done
