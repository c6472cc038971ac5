#!/bin/bash
# Winograd iteration: r5 unit tests, then stamps over the variant libraries in $LIBS.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
T=${T:-wino}
timeout -k 10 300 python -u -m pytest tests/test_gpu_r5.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/${T}_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/${T}_pytest.log
[ $rc -eq 0 ] || { tail -60 gpurun_out/${T}_pytest.log; exit $rc; }
T=${T}_st SHAPES="${SHAPES:-res32_128 res32_384 res16_256}" bash tools/wino_stamps.sh || exit 1
