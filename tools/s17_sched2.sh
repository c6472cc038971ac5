#!/bin/bash
# Round 4, session 2: linear_k32 (C5) and the attention block (C3) compiled with other AMDGPU machine schedulers.
cd "$(dirname "$0")/.." || exit 2
run() { printf '%s ' "$1"; DM_HIP_LIB=$2 timeout -k 10 200 python3 bench.py $3 --no-cpu-baseline --no-profile 2>/dev/null \
  | python3 -c "import json,sys; print(json.loads(sys.stdin.readline())['value'])" || exit 1; }
C5="--workload c5 --respace-steps 25 --steps 2 --warmup 1"
C3="--steps 3 --warmup 1"
for i in 1 2; do
  run C5_BASE "" "$C5" || exit 1
  run C5_LK_MAXILP "$PWD/tools/lib/lib_lk_maxilp.so" "$C5" || exit 1
  run C5_LK_MEMCL "$PWD/tools/lib/lib_lk_memcl.so" "$C5" || exit 1
  run C5_BASE "" "$C5" || exit 1
done
for i in 1 2; do
  run C3_BASE "" "$C3" || exit 1
  run C3_AB_MAXILP "$PWD/tools/lib/lib_ab_maxilp.so" "$C3" || exit 1
  run C3_AB_MAXILP "$PWD/tools/lib/lib_ab_maxilp.so" "$C3" || exit 1
  run C3_BASE "" "$C3" || exit 1
done
