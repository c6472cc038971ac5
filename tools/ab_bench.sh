#!/bin/bash
# A/B of two library builds in one GPU session: bench.py (no per-launch events) alternating
# the committed-HEAD build (tools/bin/libprev.so) and the working-tree build, N rounds.
cd "$(dirname "$0")/.." || exit 2
N=${N:-2}
for i in $(seq $N); do
  printf 'PREV '; DM_HIP_LIB=$PWD/tools/bin/libprev.so timeout -k 10 200 \
      python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-profile 2>/dev/null | python3 -c "import json,sys; print(json.loads(sys.stdin.readline())['value'])" || exit 1
  printf 'NEW  '; timeout -k 10 200 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-profile 2>/dev/null \
      | python3 -c "import json,sys; print(json.loads(sys.stdin.readline())['value'])" || exit 1
done
