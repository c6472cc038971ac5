#!/bin/bash
# Round 4, session 2: variant 4's software-pipelined key pass (DM_ATTN_OPT=4): bit identity, then a C3 env A/B
# in both orders.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_r4.py \
  -k "opt_variants or 8_waves" -p no:cacheprovider > gpurun_out/s7_t.log 2>&1
rc=$?; tail -3 gpurun_out/s7_t.log; [ $rc -eq 0 ] || exit $rc
VAR=DM_ATTN_OPT VAL=4 N=2 STEPS=3 bash tools/env_ab.sh
