#!/bin/bash
# Round 4, session 2: 128 x 64 linear_k32 blocks for the DiT N = 1152 GEMMs (DM_LIN_BN64): bit identity, then a
# C5 env A/B (25-step folds) in both orders.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_r4.py \
  -k "half_width or wide_blocks" -p no:cacheprovider > gpurun_out/s10_t.log 2>&1
rc=$?; tail -3 gpurun_out/s10_t.log; [ $rc -eq 0 ] || exit $rc
VAR=DM_LIN_BN64 VAL=1 N=2 STEPS=2 ARGS="--workload c5 --respace-steps 25" bash tools/env_ab.sh
