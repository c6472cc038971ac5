#!/bin/bash
# A/B of two library builds in one GPU session: bench.py (no per-launch events) alternating the
# committed-HEAD build (tools/lib/libprev.so) and the working-tree build, N rounds; ORDER=rev starts each
# round with the working tree (the chip's clock drifts over a session: check both orders). ARGS: extra
# bench.py arguments (e.g. ARGS="--workload c5 --respace-steps 25").
cd "$(dirname "$0")/.." || exit 2
N=${N:-2}
run() {  # label, lib (empty: the working tree's)
  printf '%s ' "$1"
  DM_HIP_LIB=$2 timeout -k 10 200 python3 bench.py --steps ${STEPS:-4} --warmup 1 --no-cpu-baseline --no-profile $ARGS 2>/dev/null \
      | python3 -c "import json,sys; print(json.loads(sys.stdin.readline())['value'])" || exit 1
}
for i in $(seq $N); do
  if [ "$ORDER" = rev ]; then
    run NEW "" || exit 1
    run PREV "$PWD/tools/lib/libprev.so" || exit 1
  else
    run PREV "$PWD/tools/lib/libprev.so" || exit 1
    run NEW "" || exit 1
  fi
done
