#!/bin/bash
# A/B of one build with an environment toggle: bench.py with and without VAR=VAL, N rounds, both orders.
#   VAR=DM_GN_NO_CONCAT VAL=1 N=2 bash tools/env_ab.sh
cd "$(dirname "$0")/.." || exit 2
N=${N:-2}
run() {  # label, env assignment
  printf '%s ' "$1"
  env $2 timeout -k 10 200 python3 bench.py --steps ${STEPS:-4} --warmup 1 --no-cpu-baseline --no-profile $ARGS 2>/dev/null \
      | python3 -c "import json,sys; print(json.loads(sys.stdin.readline())['value'])" || exit 1
}
for i in $(seq $N); do
  run BASE "DM_AB_NONE=1" || exit 1
  run "$VAR=$VAL" "$VAR=$VAL" || exit 1
  run "$VAR=$VAL" "$VAR=$VAL" || exit 1
  run BASE "DM_AB_NONE=1" || exit 1
done
