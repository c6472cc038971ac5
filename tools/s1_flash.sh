#!/bin/bash
# Session 2 of round 4: the 16x16x32 tail of the flash kernel's P V (Dh = 72): parity, then C5 A/B both orders.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_r3.py -k "flash or dit" tests/test_gpu_dit.py -p no:cacheprovider > gpurun_out/s1_flash_t.log 2>&1
rc=$?; tail -3 gpurun_out/s1_flash_t.log; [ $rc -eq 0 ] || exit $rc
ARGS="--workload c5 --respace-steps 25" STEPS=2 N=1 bash tools/ab_bench.sh || exit 1
ORDER=rev ARGS="--workload c5 --respace-steps 25" STEPS=2 N=1 bash tools/ab_bench.sh || exit 1
