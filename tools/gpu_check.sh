#!/bin/bash
# One GPU session: parity tests, smoke, short bench. Every GPU step has its own
# time limit; a crash/abort/timeout (exit >= 124 or signal) ends the script.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
step() {  # name, timeout, command...
  local name=$1 lim=$2; shift 2
  echo "== $name" ; date
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 30 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -gt 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-}
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python -u bench.py --steps ${BENCH_STEPS:-2} --warmup 1 --profile-json gpurun_out/bench_profile.json
