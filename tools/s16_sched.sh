#!/bin/bash
# Round 4, session 2: the K32 conv compiled with other AMDGPU machine schedulers (same arithmetic, bit-identical
# by construction): C3 bench alternating the tree's library with tools/lib/lib_max-ilp.so and lib_max-memory-clause.so.
cd "$(dirname "$0")/.." || exit 2
run() { printf '%s ' "$1"; DM_HIP_LIB=$2 timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile 2>/dev/null \
  | python3 -c "import json,sys; print(json.loads(sys.stdin.readline())['value'])" || exit 1; }
for i in 1 2; do
  run BASE "" || exit 1
  run MAXILP "$PWD/tools/lib/lib_max-ilp.so" || exit 1
  run MEMCL "$PWD/tools/lib/lib_max-memory-clause.so" || exit 1
  run MEMCL "$PWD/tools/lib/lib_max-memory-clause.so" || exit 1
  run MAXILP "$PWD/tools/lib/lib_max-ilp.so" || exit 1
  run BASE "" || exit 1
done
