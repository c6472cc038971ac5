#!/bin/bash
# K32 conv iteration loop on the GPU box: exact/accuracy tests of conv_k32, then the CIFAR conv shapes
# with conv_patch3 (tile 4) and conv_k32 (tile 10) side by side.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_k32.py -x -q --timeout 120 --timeout-method thread > gpurun_out/k32_tests.log 2>&1
rc=$?; tail -3 gpurun_out/k32_tests.log; [ $rc -ne 0 ] && exit $rc
for s in ${SHAPES:-res32_128 res32_256 res16_256}; do
  timeout -k 10 120 python -u tools/conv_bench.py --shape $s --math fp16x2 --tiles ${TILES:-4,10} --iters 30 || exit $?
done
