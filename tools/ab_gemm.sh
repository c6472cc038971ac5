#!/bin/bash
# A/B of the GEMM microbenchmark: committed-HEAD build (tools/bin/libprev.so) vs the working tree.
cd "$(dirname "$0")/.." || exit 2
PREV=$PWD/tools/bin/libprev.so
DM_HIP_LIB=$PREV timeout -k 10 120 python -u tools/gemm_bench.py 2>&1 | grep fp16x2 | sed "s/^/PREV /" || exit 1
timeout -k 10 120 python -u tools/gemm_bench.py 2>&1 | grep fp16x2 | sed "s/^/NEW  /" || exit 1
