#!/bin/bash
# Round-4 kernel-trace + FETCH / WRITE PMC profiles of the C4 and C5 benches (10-step folds in the trace).
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
WORKLOAD=c5 STEPS=10 TAG=r04_v1_c5 bash tools/gpu_profile.sh > gpurun_out/prof_c5.out 2>&1 || { tail -20 gpurun_out/prof_c5.out; exit 1; }
tail -12 gpurun_out/prof_c5.out
WORKLOAD=c4 STEPS=10 TAG=r04_v1_c4 bash tools/gpu_profile.sh > gpurun_out/prof_c4.out 2>&1 || { tail -20 gpurun_out/prof_c4.out; exit 1; }
tail -12 gpurun_out/prof_c4.out
