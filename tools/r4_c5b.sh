#!/bin/bash
# C5: the 8-wave 128 x 256 linear_k32 blocks -- bit-identity test, then same-box A/B (25-step folds).
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_r4.py -m gpu -q -x -k "wide_blocks" --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_c5b.log 2>&1 || { tail -30 gpurun_out/pytest_c5b.log; exit 1; }
tail -2 gpurun_out/pytest_c5b.log
for w in ${WIDES:-1 2}; do
  echo "== DM_LIN_BN256=$w"
  VAR=DM_LIN_BN256 VAL=$w N=1 STEPS=3 ARGS="--workload c5 --respace-steps 25" bash tools/env_ab.sh || exit 1
done
