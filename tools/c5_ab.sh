cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dit.py > gpurun_out/dit_t.log 2>&1; rc=$?; tail -2 gpurun_out/dit_t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for e in 1 0; do
  printf "presplit=$e "
  DM_DIT_PRESPLIT=$e timeout -k 10 200 python3 bench.py --workload c5 --steps 2 --warmup 1 --respace-steps 25 --no-cpu-baseline --no-profile 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'])" || exit 1
done; done
