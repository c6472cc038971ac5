#!/bin/bash
# Winograd iteration: unit tests, bench A/B vs the direct conv, per-op profiles of both arms.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
T=${T:-r5_w2}
timeout -k 10 300 python -u -m pytest tests/test_gpu_r5.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/${T}_pytest.log 2>&1
rc=$?
tail -5 gpurun_out/${T}_pytest.log
[ $rc -eq 0 ] || exit $rc
VAR=DM_CONV_WINO VAL=0 N=${N:-2} STEPS=4 bash tools/env_ab.sh 2>&1 | tee gpurun_out/${T}_ab.txt || exit 1
timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --profile-json gpurun_out/${T}_prof_wino.json > gpurun_out/${T}_bench_wino.json || exit 1
DM_CONV_WINO=0 timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --profile-json gpurun_out/${T}_prof_direct.json > gpurun_out/${T}_bench_direct.json || exit 1
