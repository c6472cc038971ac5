#!/bin/bash
# Winograd tile order (column halves outer at every map size): Winograd / forward tests, then C3 A/B against the
# HEAD build (tools/lib/libprev.so), both orders.
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_r5.py tests/test_gpu_r6.py tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t17.log 2>&1
rc=$?; tail -3 gpurun_out/t17.log; [ $rc -eq 0 ] || exit $rc
N=2 bash tools/ab_bench.sh > gpurun_out/ab_order_a.txt 2>&1 || exit 1
N=2 ORDER=rev bash tools/ab_bench.sh > gpurun_out/ab_order_b.txt 2>&1 || exit 1
cat gpurun_out/ab_order_a.txt gpurun_out/ab_order_b.txt
