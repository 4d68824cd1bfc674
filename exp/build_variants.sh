#!/bin/bash
# experiment builds of libhonk_hip.so with -D flags (not part of the product)
set -e
cd "$(dirname "$0")/.."
for v in "$@"; do
  name=${v%%=*}; flags=${v#*=}
  mkdir -p exp/$name
  for src in runtime.cpp res.hip cnn.hip train.hip mfcc.hip; do
    x=""; [[ $src == *.cpp ]] && x="-x hip"
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $flags $x -c honk_amd/csrc/$src -o exp/$name/${src%.*}.o &
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o exp/$name/libhonk_hip.so exp/$name/*.o
done
