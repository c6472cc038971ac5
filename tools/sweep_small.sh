#!/bin/bash
# Forced-tile sweep of the CIFAR conv shapes (tools/conv_bench.py; tiles that do not take a shape print n/a)
cd "$(dirname "$0")/.." || exit 2
for s in ${SHAPES:-res8_256 res8_512 res16_256 res32_256 res32_128 res32_384 up16_256}; do
  timeout -k 10 90 python3 -u tools/conv_bench.py --shape $s --math fp16x2 --tiles ${TILES:-0,16} --iters 50 2>&1 | grep -v amdgpu.ids || exit 1
done
