#!/bin/bash
# Wide-map Winograd iteration: its tests (+ the round-5 Winograd tests), then C4 A/B pairs (5-step folds) of the
# committed build (tools/lib/libprev.so) against the working tree, both orders.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_r6.py tests/test_gpu_r5.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/wide_pytest.log 2>&1 || { tail -60 gpurun_out/wide_pytest.log; exit 1; }
tail -3 gpurun_out/wide_pytest.log
N=${N:-1} ARGS="--workload c4 --respace-steps 5" bash tools/ab_bench.sh && \
  N=${N:-1} ORDER=rev ARGS="--workload c4 --respace-steps 5" bash tools/ab_bench.sh
