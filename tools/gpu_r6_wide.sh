#!/bin/bash
# Wide-map Winograd tile order: the wide / ADM tests, then C4 A/B against the HEAD build (tools/lib/libprev.so), both
# orders, 20 respaced steps.
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_r6.py tests/test_gpu_adm.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/t16.log 2>&1
rc=$?; tail -3 gpurun_out/t16.log; [ $rc -eq 0 ] || exit $rc
N=2 STEPS=1 ARGS="--workload c4 --respace-steps 20" bash tools/ab_bench.sh > gpurun_out/ab_wide_a.txt 2>&1 || exit 1
N=2 STEPS=1 ORDER=rev ARGS="--workload c4 --respace-steps 20" bash tools/ab_bench.sh > gpurun_out/ab_wide_b.txt 2>&1 || exit 1
cat gpurun_out/ab_wide_a.txt gpurun_out/ab_wide_b.txt
