#!/bin/bash
# Winograd iteration: unit tests, conv microbench (direct vs wino), stamps, bench A/B, per-op profiles.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
T=${T:-r5_w3}
timeout -k 10 300 python -u -m pytest tests/test_gpu_r5.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/${T}_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/${T}_pytest.log
[ $rc -eq 0 ] || exit $rc
for sh in res32_128 res32_256 res32_384 res16_256; do
  timeout -k 10 120 python3 tools/conv_bench.py --shape $sh --math fp16x2 --tiles 10,21 --iters 20 || exit 1
done 2>&1 | tee gpurun_out/${T}_convbench.txt
for sh in res32_128 res32_384 res16_256; do
  DM_HIP_LIB=tools/stampslib/libdm_stamps.so timeout -k 10 120 python3 tools/wino_stamps.py --shape $sh || exit 1
done 2>&1 | tee gpurun_out/${T}_stamps.txt
VAR=DM_CONV_WINO VAL=0 N=${N:-2} STEPS=4 bash tools/env_ab.sh 2>&1 | tee gpurun_out/${T}_ab.txt || exit 1
timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --profile-json gpurun_out/${T}_prof_wino.json > gpurun_out/${T}_bench_wino.json || exit 1
