#!/bin/bash
# Round 4, session 2: C3 kernel trace + FETCH / WRITE PMC of the final build (tools/gpu_profile.sh).
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
TAG=r04_v3 bash tools/gpu_profile.sh > gpurun_out/prof_c3.out 2>&1; rc=$?; tail -30 gpurun_out/prof_c3.out; exit $rc
