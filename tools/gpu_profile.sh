#!/bin/bash
# rocprofv3 kernel-trace summary + separate PMC passes (FETCH_SIZE, WRITE_SIZE) of bench.py.
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
TAG=${TAG:-r01}
mkdir -p gpurun_out
run() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?;
        echo "== $name rc=$rc"; tail -n 5 "gpurun_out/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run prof_stats 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o trace -- \
    python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline
if [ -z "$NO_PMC" ]; then
run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch_$TAG -o fetch -- \
    python3 bench.py --steps 1 --warmup 0 --respace-steps 2 --no-cpu-baseline
run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write_$TAG -o write -- \
    python3 bench.py --steps 1 --warmup 0 --respace-steps 2 --no-cpu-baseline
fi
find gpurun_out -name "*.csv" | head -20
