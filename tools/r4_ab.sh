#!/bin/bash
# Round-4 measurement batch on the box: attention-block phase stamps (v2 / v3), then same-box env A/B pairs.
#   gpurun --timeout 1200 -- 'bash tools/r4_ab.sh'
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
for v in 3 2; do
  DM_ATTN_BLOCK=$v DM_HIP_LIB=tools/lib/libdm_stamps.so timeout -k 10 150 python3 tools/ab_stamps.py \
    > gpurun_out/stamps_v$v.txt 2>&1 || { tail -5 gpurun_out/stamps_v$v.txt; exit 1; }
  tail -12 gpurun_out/stamps_v$v.txt
done
for pair in ${PAIRS:-DM_ATTN_BLOCK=2 DM_ATTN_FOLD=0 DM_K32S_W4=1}; do
  VAR=${pair%%=*} VAL=${pair#*=} N=${N:-1} bash tools/env_ab.sh > gpurun_out/ab_${pair}.txt 2>&1 || { cat gpurun_out/ab_${pair}.txt; exit 1; }
  echo "== $pair"; cat gpurun_out/ab_${pair}.txt
done
