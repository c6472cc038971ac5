#!/bin/bash
# Round 4, session 2, last build (8^2 single-image tiles default): the whole GPU suite, smoke(), the C3 line.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests -p no:cacheprovider \
  > gpurun_out/s18_suite.log 2>&1; rc=$?; tail -2 gpurun_out/s18_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s18_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/s18_smoke.log
timeout -k 10 300 python3 bench.py > gpurun_out/s18_bench_c3.json 2> gpurun_out/s18_bench_c3.err || exit 1
cut -c1-300 gpurun_out/s18_bench_c3.json
