#!/bin/bash
# 4 x 4 Winograd iteration on one GPU box: its tests (+ the forwards that route the 4^2 level through it), the conv
# microbenchmark (conv_k32s, tile 15, vs the split-K Winograd kernel, tile 21, at 2 / 4 splits), then C3 A/B pairs
# of the committed build (tools/lib/libprev.so) against the working tree, both orders.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
T=${T:-w4}
timeout -k 10 600 python -u -m pytest tests/test_gpu_r6.py tests/test_gpu_r3.py::test_small_map_conv_vs_splitk \
  tests/test_gpu_r5.py::test_wino_cifar_forward tests/test_gpu_r5.py::test_small_map_variants_both_launched_bit_identical \
  ${EXTRA_TESTS} -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 \
  || { tail -60 gpurun_out/${T}_pytest.log; exit 1; }
tail -3 gpurun_out/${T}_pytest.log
for s in ${SHAPES-res4_256 res4_512}; do
  timeout -k 10 120 python -u tools/conv_bench.py --shape $s --math fp16x2 --tiles 15 --ksplit 2 --iters 40 || exit 1
  for k in 2 4; do
    timeout -k 10 120 python -u tools/conv_bench.py --shape $s --math fp16x2 --tiles 21 --ksplit $k --iters 40 || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${T}_conv.txt
if [ "${N:-2}" -gt 0 ]; then
  { N=${N:-2} bash tools/ab_bench.sh && N=${N:-2} ORDER=rev bash tools/ab_bench.sh; } | tee gpurun_out/${T}_c3.txt
fi
