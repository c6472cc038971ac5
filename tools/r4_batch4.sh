#!/bin/bash
# Round-4 batch 4: attention variant 5 tests, per-family profile and same-box A/B against the default (4).
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_r4.py -m gpu -q -x -k "folded" --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_b4.log 2>&1 || { tail -30 gpurun_out/pytest_b4.log; exit 1; }
tail -2 gpurun_out/pytest_b4.log
DM_ATTN_BLOCK=5 timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline \
  --profile-json gpurun_out/c3_prof_v5.json > gpurun_out/bench_v5.json 2>gpurun_out/bench_v5.err || { tail gpurun_out/bench_v5.err; exit 1; }
python3 tools/prof_top.py gpurun_out/c3_prof_v5.json 6
VAR=DM_ATTN_BLOCK VAL=5 N=1 bash tools/env_ab.sh
