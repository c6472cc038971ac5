#!/bin/bash
# Round-6 small-kernel check on one GPU box: the attention / GEMM / forward tests, env A/Bs of the small-map attention
# block and the time-MLP linear_rows, and a short kernel trace of the kernels they touch (tools/trace_top.py).
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_r6.py tests/test_gpu_r4.py tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t6.log 2>&1; rc=$?; tail -3 gpurun_out/t6.log
[ $rc -eq 0 ] || exit $rc
for v in DM_ATTN_SMALL DM_LIN_ROWS; do
  echo "== $v"; VAR=$v VAL=0 N=2 bash tools/env_ab.sh > gpurun_out/ab_$v.txt 2>&1 || exit 1; cat gpurun_out/ab_$v.txt
done
rm -rf gpurun_out/prof6
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof6 -o t -- python3 bench.py --steps 1 --warmup 1 \
  --respace-steps 5 --no-cpu-baseline --no-profile > gpurun_out/prof6.log 2>&1 || exit 1
python3 tools/trace_top.py "$(find gpurun_out/prof6 -name '*.db' | head -1)" small_out linear_rows attn_small gemm_kernel small_in
rm -rf gpurun_out/prof6
