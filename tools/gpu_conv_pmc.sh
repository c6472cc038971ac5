#!/bin/bash
# Conv microbenchmark + one SQ PMC pass over one conv shape (MATH selects the kernel family).
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
SHAPE=${SHAPE:-res32_256}
MATH=${MATH:-bf16x3}
timeout -k 10 300 python3 tools/conv_bench.py > gpurun_out/conv_bench.log 2>&1 || exit $?
cat gpurun_out/conv_bench.log
if [ -n "$PMC" ]; then
  timeout -s KILL 90 rocprofv3 --pmc $PMC --kernel-trace -d gpurun_out/conv_pmc -o pmc -- \
      python3 tools/conv_bench.py --shape $SHAPE --math $MATH --iters 5 > gpurun_out/conv_pmc.log 2>&1 || exit $?
  tail -3 gpurun_out/conv_pmc.log
fi
