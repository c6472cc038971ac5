#!/bin/bash
# Round 4, session 2, last build: the C5 / C2 / C4 bench lines (one fold each).
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
for w in c5 c2 c4; do
  timeout -k 10 400 python3 bench.py --workload $w --steps 1 --warmup 0 > gpurun_out/s15_bench_$w.json 2> gpurun_out/s15_bench_$w.err || exit 1
  cut -c1-200 gpurun_out/s15_bench_$w.json
done
