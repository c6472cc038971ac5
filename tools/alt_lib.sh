#!/bin/bash
# Alternative library with one source recompiled under extra flags (A/B of kernel variants):
#   bash tools/alt_lib.sh <source.hip> <out.so> <flags...>
# links the rest of the current build's objects (make first).
set -e
cd "$(dirname "$0")/../diffusion-models-pytorch_amd/csrc"
src=$1; out=$2; shift 2
mkdir -p build_alt
obj=build_alt/$(basename $out .so)_${src%.hip}.o
extra=""
[ "$src" = conv_wino.hip ] && extra="-fno-slp-vectorize"   # as the Makefile builds it
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-function \
  -Wno-unused-variable -I../../include $extra "$@" -c $src -o $obj
objs=$(ls build/*.o | grep -v "build/${src%.hip}.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out $objs $obj -ldl
