#!/bin/bash
# Round-4 batch 6: N-slow tile order of the 2-D tiles (tests under DM_K32_NSLOW=1, C4 A/B), attention S prefetch A/B.
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
DM_K32_NSLOW=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_r4.py -m gpu -q -x -k "t2d" --timeout 250 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_b6.log 2>&1 || { tail -30 gpurun_out/pytest_b6.log; exit 1; }
tail -2 gpurun_out/pytest_b6.log
VAR=DM_K32_NSLOW VAL=1 N=1 STEPS=1 ARGS="--workload c4 --respace-steps 10" bash tools/env_ab.sh || exit 1
bash tools/r4_batch5.sh
