#!/bin/bash
# A/B of the conv microbenchmark: committed-HEAD build (tools/bin/libprev.so) vs the working tree.
cd "$(dirname "$0")/.." || exit 2
PREV=$PWD/tools/bin/libprev.so
for s in ${SHAPES:-res32_128 res32_256 res16_256 up16_256 qkv16}; do
  DM_HIP_LIB=$PREV timeout -k 10 60 python -u tools/conv_bench.py --shape $s --math fp16x2 2>&1 | grep -v amdgpu.ids | sed "s/^/PREV /" || exit 1
  timeout -k 10 60 python -u tools/conv_bench.py --shape $s --math fp16x2 2>&1 | grep -v amdgpu.ids | sed "s/^/NEW  /" || exit 1
done
