#!/bin/bash
# The last conv's in-kernel GroupNorm finalize: forward / sampler tests, then a short kernel trace of the last conv and
# the finalize launches (tools/trace_top.py).
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_r6.py tests/test_gpu_ops.py tests/test_gpu_samplers.py \
  tests/test_gpu_r3.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t8.log 2>&1
rc=$?; tail -3 gpurun_out/t8.log; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/prof8
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof8 -o t -- python3 bench.py --steps 1 --warmup 1 \
  --respace-steps 5 --no-cpu-baseline --no-profile > gpurun_out/prof8.log 2>&1 || exit 1
python3 tools/trace_top.py "$(find gpurun_out/prof8 -name '*.db' | head -1)" small_out gn_finalize attn_small linear_rows
rm -rf gpurun_out/prof8
