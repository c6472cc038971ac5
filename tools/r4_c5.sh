#!/bin/bash
# C5 (DiT-XL/2 DDIMCFG) same-box A/B of the linear_k32 tile-order group size (DM_LIN_GM, default 4).
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
for gm in ${GMS:-8 16}; do
  echo "== DM_LIN_GM=$gm"
  VAR=DM_LIN_GM VAL=$gm N=1 STEPS=3 ARGS="--workload c5 --respace-steps 25" bash tools/env_ab.sh || exit 1
done
