#!/bin/bash
# Round 4, session 2, final build: the whole GPU suite + smoke, then the working tree against the committed HEAD
# (tools/lib/libprev.so) in both orders (the in-kernel finalize's concat branch must not cost the default path).
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests -p no:cacheprovider \
  > gpurun_out/s13_suite.log 2>&1; rc=$?; tail -2 gpurun_out/s13_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s13_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/s13_smoke.log
N=2 STEPS=3 bash tools/ab_bench.sh || exit 1
ORDER=rev N=1 STEPS=3 bash tools/ab_bench.sh || exit 1
