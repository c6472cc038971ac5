#!/bin/bash
# Round 4, session 2: C5 kernel trace + FETCH / WRITE PMC of the flash-tail build, and the C5 bench line.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
WORKLOAD=c5 STEPS=10 TAG=r04_v2_c5 bash tools/gpu_profile.sh > gpurun_out/prof_c5.out 2>&1 || { tail -20 gpurun_out/prof_c5.out; exit 1; }
tail -12 gpurun_out/prof_c5.out
timeout -k 10 400 python3 bench.py --workload c5 --steps 1 --warmup 0 > gpurun_out/s3_bench_c5.json 2> gpurun_out/s3_bench_c5.err || exit 1
cut -c1-300 gpurun_out/s3_bench_c5.json
