#!/bin/bash
# Winograd kernel iteration on one GPU box: its parity tests, the conv microbenchmark (HEAD build in
# tools/lib/libprev.so vs the working tree, tile 21 = conv_wino), then C3 A/B pairs in both orders.
#   TESTS="tests/test_gpu_r5.py" SHAPES="res32_128 res16_256" N=1 bash tools/gpu_wino_ab.sh
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
T=${T:-wino_ab}
if [ -n "${TESTS-tests/test_gpu_r5.py}" ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS-tests/test_gpu_r5.py} -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
  tail -3 gpurun_out/${T}_pytest.log
fi
for s in ${SHAPES-res32_128 res32_384 res32_256 res16_256 res8_256 res8_512}; do
  for lib in "$PWD/tools/lib/libprev.so" ""; do
    tag=NEW; [ -n "$lib" ] && tag=PREV
    DM_HIP_LIB=$lib timeout -k 10 90 python -u tools/conv_bench.py --shape $s --math fp16x2 --tiles 21 --iters 40 2>&1 \
      | grep -v amdgpu.ids | sed "s/^/$tag /" || exit 1
  done
done | tee gpurun_out/${T}_conv.txt
if [ "${N:-2}" -gt 0 ]; then
  { N=${N:-2} bash tools/ab_bench.sh && N=${N:-2} ORDER=rev bash tools/ab_bench.sh; } | tee gpurun_out/${T}_c3.txt
fi
