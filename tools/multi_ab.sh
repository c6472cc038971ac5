#!/bin/bash
# A/B/C/... of one build over several environment settings: bench.py once per setting per round, N rounds,
# the order reversed on every other round.
#   CFGS="DM_AB_NONE=1 DM_LIN_SK=0" N=2 STEPS=1 ARGS="--workload c5 --respace-steps 25" bash tools/multi_ab.sh
cd "$(dirname "$0")/.." || exit 2
N=${N:-2}
read -r -a cfgs <<< "$CFGS"
run() {
  printf '%s ' "$1"
  env $1 timeout -k 10 200 python3 bench.py --steps ${STEPS:-4} --warmup 1 --no-cpu-baseline --no-profile $ARGS 2>/dev/null \
      | python3 -c "import json,sys; print(json.loads(sys.stdin.readline())['value'])" || exit 1
}
for i in $(seq $N); do
  if [ $((i % 2)) -eq 1 ]; then order=("${cfgs[@]}"); else order=(); for ((k=${#cfgs[@]}-1; k>=0; k--)); do order+=("${cfgs[$k]}"); done; fi
  for c in "${order[@]}"; do run "$c" || exit 1; done
done
