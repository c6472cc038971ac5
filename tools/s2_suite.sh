#!/bin/bash
# Round 4, session 2: the C-ABI gather test, the whole GPU suite, the C3 bench line.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_comm.py -p no:cacheprovider \
  > gpurun_out/s2_comm.log 2>&1; rc=$?; tail -4 gpurun_out/s2_comm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 800 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests -p no:cacheprovider \
  > gpurun_out/s2_suite.log 2>&1; rc=$?; tail -2 gpurun_out/s2_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py > gpurun_out/s2_bench_c3.json 2> gpurun_out/s2_bench_c3.err || exit 1
cut -c1-300 gpurun_out/s2_bench_c3.json
