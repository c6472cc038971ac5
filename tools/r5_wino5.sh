#!/bin/bash
# Winograd iteration: unit tests, stamps, bench A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
T=${T:-r5_w5}
timeout -k 10 300 python -u -m pytest tests/test_gpu_r5.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/${T}_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/${T}_pytest.log
[ $rc -eq 0 ] || { tail -60 gpurun_out/${T}_pytest.log; exit $rc; }
cp gpurun_out/parity_report.json gpurun_out/${T}_parity.json
T=${T}_st LIBS="tools/stampslib/libdm_stamps.so $XLIBS" SHAPES="res32_128 res32_384 res16_256" bash tools/r5_stamps.sh || exit 1
VAR=DM_CONV_WINO VAL=0 N=${N:-2} STEPS=4 bash tools/env_ab.sh 2>&1 | tee gpurun_out/${T}_ab.txt || exit 1
