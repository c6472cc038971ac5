#!/bin/bash
# Round-4 batch 7: 8^2 single-image tiles (DM_K32_8X=1): bit-identity test and C3 A/B.
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_r4.py -m gpu -q -x -k "8x8" --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_b7.log 2>&1 || { tail -30 gpurun_out/pytest_b7.log; exit 1; }
tail -2 gpurun_out/pytest_b7.log
VAR=DM_K32_8X VAL=1 N=2 bash tools/env_ab.sh
