#!/bin/bash
# Round 4, session 2: concat GroupNorm statistics combined in the consumer conv (no gn_concat_stats launch):
# bit identity + the GN toggles + the parity suite's forwards, then a C3 env A/B in both orders.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_r4.py \
  tests/test_gpu_presplit.py tests/test_gpu_parity.py tests/test_gpu_adagn.py -p no:cacheprovider > gpurun_out/s12_t.log 2>&1
rc=$?; tail -3 gpurun_out/s12_t.log; [ $rc -eq 0 ] || exit $rc
VAR=DM_GN_CONCAT_LAUNCH VAL=1 N=2 STEPS=3 bash tools/env_ab.sh
