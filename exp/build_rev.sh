#!/bin/bash
# experiment build of libhonk_hip.so from a git revision: exp/build_rev.sh <name> <rev>
set -e
cd "$(dirname "$0")/.."
name=$1; rev=$2
mkdir -p exp/$name/src/csrc exp/$name/include
for f in $(git ls-tree --name-only $rev honk_amd/csrc/); do git show $rev:$f > exp/$name/src/csrc/$(basename $f); done
git show $rev:include/honk_hip.h > exp/$name/include/honk_hip.h
mkdir -p exp/$name/src/include; cp exp/$name/include/honk_hip.h exp/$name/src/include/
for src in runtime.cpp res.hip cnn.hip train.hip mfcc.hip; do
  x=""; [[ $src == *.cpp ]] && x="-x hip"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $x -c exp/$name/src/csrc/$src -o exp/$name/${src%.*}.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o exp/$name/libhonk_hip.so exp/$name/*.o
