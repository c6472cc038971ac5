#!/bin/bash
# GPU box: secondary-workload benches (BASELINE configs C2 / C4 / C5) after the headline C3 line.
# Each step has its own limit; a crash / abort / timeout ends the script.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
step() {  # name, timeout, command...
  local name=$1 lim=$2; shift 2
  echo "== $name"; date
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
for w in ${WORKLOADS:-c5 c2}; do
  step bench_$w ${WL_TIMEOUT:-600} python -u bench.py --workload $w --steps 1 --warmup 0 \
    --profile-json gpurun_out/bench_${w}_profile.json $BENCH_ARGS
done
