#!/bin/bash
# C4 (ADM-256 UNetCombined DDIMCFG) same-box A/B of the wide-map 2-D tiles (DM_CONV_K32T2=0: 128-pixel row
# segments), 10 respaced steps per fold, plus the t2d test.
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_r4.py -m gpu -q -x -k "adm256_t2d" --timeout 250 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_c4.log 2>&1 || { tail -30 gpurun_out/pytest_c4.log; exit 1; }
tail -2 gpurun_out/pytest_c4.log
VAR=DM_CONV_K32T2 VAL=0 N=1 STEPS=1 ARGS="--workload c4 --respace-steps 10" bash tools/env_ab.sh
