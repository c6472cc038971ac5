#!/bin/bash
# Round-2 closing measurements: GPU suite, bench lines of C3 (default args, with the CPU baseline), C2, C4,
# C5, then the C3 kernel-trace + PMC profile (tools/gpu_profile.sh). Outputs under gpurun_out/.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests > gpurun_out/suite_final.log 2>&1
rc=$?; tail -2 gpurun_out/suite_final.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || exit 1
cat gpurun_out/bench_c3.json
for w in c2 c5 c4; do
  timeout -k 10 400 python3 bench.py --workload $w --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || exit 1
  cat gpurun_out/bench_$w.json
done
TAG=${TAG:-r02_v7} bash tools/gpu_profile.sh > gpurun_out/prof_final.out 2>&1; rc=$?; tail -25 gpurun_out/prof_final.out; exit $rc
