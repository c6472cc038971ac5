#!/bin/bash
# GPU test run on the box: the round-3 tests first, then the whole -m gpu suite.
#   gpurun --timeout 1200 -- '[K=<-k expression>] bash tools/gpu_tests.sh [pytest-selection]'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
sel=${1:-tests}
timeout -k 10 1100 python -u -m pytest $sel ${K:+-k "$K"} -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest.log 2>&1
rc=$?
tail -30 gpurun_out/pytest.log
exit $rc
