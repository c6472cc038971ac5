#!/bin/bash
# conv_bench of SHAPES (ksplit KS, tiles TILES) with the committed-HEAD build (tools/bin/libprev.so) and the
# working tree's, alternating, N rounds
cd "$(dirname "$0")/.." || exit 2
for i in $(seq ${N:-2}); do
  for lib in "$PWD/tools/bin/libprev.so" ""; do
    for s in ${SHAPES:-res4_256 res4_512}; do
      printf '%s ' "${lib:+PREV}${lib:-NEW}"
      DM_HIP_LIB=$lib timeout -k 10 60 python3 -u tools/conv_bench.py --shape $s --math fp16x2 --tiles ${TILES:-0} \
          --ksplit ${KS:-2} --iters 100 2>&1 | grep -v amdgpu.ids || exit 1
    done
  done
done
