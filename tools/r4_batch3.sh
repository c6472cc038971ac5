#!/bin/bash
# Round-4 batch 3: deferred-range repack test, v3 / v4 attention per-family profiles, v4 A/B, C5 tile order A/B.
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_r3.py -m gpu -q -x -k "deferred" --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_b3.log 2>&1 || { tail -30 gpurun_out/pytest_b3.log; exit 1; }
tail -2 gpurun_out/pytest_b3.log
for v in 3 4; do
  DM_ATTN_BLOCK=$v timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline \
    --profile-json gpurun_out/c3_prof_v$v.json > gpurun_out/bench_v$v.json 2>gpurun_out/bench_v$v.err || { tail gpurun_out/bench_v$v.err; exit 1; }
  echo "== v$v"; python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_v$v.json').readline()); print(d['value'])"
  python3 tools/prof_top.py gpurun_out/c3_prof_v$v.json 8
done
VAR=DM_ATTN_BLOCK VAL=4 N=1 bash tools/env_ab.sh || exit 1
[ -n "$NO_C5" ] || bash tools/r4_c5.sh
