#!/bin/bash
# Alternate bench.py over several library builds in one GPU session (same box): LIBS="a.so b.so ..." (paths
# relative to the repo; "" = the working tree's), N rounds, ARGS extra bench arguments.
cd "$(dirname "$0")/.." || exit 2
for i in $(seq ${N:-2}); do
  for L in $LIBS; do
    [ "$L" = tree ] && L=""
    printf '%s ' "${L:-tree}"
    DM_HIP_LIB=${L:+$PWD/$L} timeout -k 10 200 python3 bench.py --steps ${STEPS:-4} --warmup 1 --no-cpu-baseline --no-profile $ARGS 2>/dev/null \
        | python3 -c "import json,sys; print(json.loads(sys.stdin.readline())['value'])" || exit 1
  done
done
