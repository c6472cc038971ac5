#!/bin/bash
# scratch GPU iteration: optional conv sweep, the given test files, then an A/B bench against tools/bin/libprev.so
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
if [ -n "$SWEEP" ]; then bash tools/sweep_small.sh > gpurun_out/sweep.log 2>&1 || { cat gpurun_out/sweep.log; exit 1; }; cat gpurun_out/sweep.log; fi
timeout -k 10 500 python -u -m pytest -x -q ${TESTS:-tests/test_gpu_parity.py} --timeout 200 --timeout-method thread > gpurun_out/par.log 2>&1; rc=$?; tail -3 gpurun_out/par.log; [ $rc -eq 0 ] || exit $rc
N=${N:-2} bash tools/ab_bench.sh
