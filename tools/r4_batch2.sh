#!/bin/bash
# Round-4 batch: stride-2 K32 tests, per-family profiles of v2 / v3 attention, stride-2 A/B.
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_r4.py tests/test_gpu_conv_split.py tests/test_gpu_ops.py -m gpu -q -x \
  -k "stride2 or downsample or conv3x3_exact" --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_b2.log 2>&1 || { tail -30 gpurun_out/pytest_b2.log; exit 1; }
tail -3 gpurun_out/pytest_b2.log
for v in 2 3; do
  DM_ATTN_BLOCK=$v timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline \
    --profile-json gpurun_out/c3_prof_v$v.json > gpurun_out/bench_v$v.json 2>gpurun_out/bench_v$v.err || { tail gpurun_out/bench_v$v.err; exit 1; }
  echo "== v$v"; cat gpurun_out/bench_v$v.json | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['roofline'])"
  python3 tools/prof_top.py gpurun_out/c3_prof_v$v.json 16
done
VAR=DM_CONV_K32S2 VAL=0 N=1 bash tools/env_ab.sh
