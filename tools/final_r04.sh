#!/bin/bash
# Round-4 measurements, part 1 (STAGE=suite): the GPU suite and the C3 bench line (default arguments, with
# the CPU baseline); part 2 (STAGE=lines): the C2 / C4 / C5 lines and the C3 kernel-trace + PMC profile
# (tools/gpu_profile.sh, TAG). Outputs under gpurun_out/.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
if [ "${STAGE:-suite}" = suite ]; then
  timeout -k 10 800 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests > gpurun_out/suite_final.log 2>&1
  rc=$?; tail -2 gpurun_out/suite_final.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python3 bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || exit 1
  cat gpurun_out/bench_c3.json
  exit 0
fi
for w in c5 c2 c4; do
  timeout -k 10 400 python3 bench.py --workload $w --steps 1 --warmup 0 > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || exit 1
  cut -c1-400 gpurun_out/bench_$w.json
done
TAG=${TAG:-r04_v1} bash tools/gpu_profile.sh > gpurun_out/prof_final.out 2>&1; rc=$?; tail -25 gpurun_out/prof_final.out; exit $rc
