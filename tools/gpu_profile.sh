#!/bin/bash
# rocprofv3 kernel-trace summary + separate PMC passes (FETCH_SIZE, WRITE_SIZE) of bench.py, then the
# committed summaries (profiles/<TAG>_kernel_stats.csv, profiles/<TAG>_pmc.json).
#   TAG=r02_v1 [WORKLOAD=c3|c2|c4|c5] [STEPS=<respaced steps of the traced fold>] bash tools/gpu_profile.sh
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
TAG=${TAG:-r02}
WL=${WORKLOAD:-c3}
mkdir -p gpurun_out
run() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?;
        echo "== $name rc=$rc"; tail -n 5 "gpurun_out/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
SARGS=""
[ -n "$STEPS" ] && SARGS="--respace-steps $STEPS"
BENCH="bench.py --workload $WL --no-cpu-baseline"
run prof_$TAG 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o trace -- \
    python3 $BENCH --steps 1 --warmup 1 $SARGS
if [ -z "$NO_PMC" ]; then
run pmc_fetch_$TAG 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch_$TAG -o fetch -- \
    python3 $BENCH --steps 1 --warmup 0 --respace-steps 2
run pmc_write_$TAG 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write_$TAG -o write -- \
    python3 $BENCH --steps 1 --warmup 0 --respace-steps 2
BUILD=$(python3 -c "import sys; sys.path.insert(0, 'diffusion-models-pytorch_amd'); import dmhip; print(dmhip.build_info())")
python3 tools/rocpd_report.py --tag $TAG --workload $WL --build "$BUILD" \
    --trace "$(find gpurun_out/prof_$TAG -name 'trace_results.db' | head -n 1)" \
    --fetch "$(find gpurun_out/pmc_fetch_$TAG -name 'fetch_results.db' | head -n 1)" \
    --write "$(find gpurun_out/pmc_write_$TAG -name 'write_results.db' | head -n 1)" \
    --command "rocprofv3 --pmc FETCH_SIZE|WRITE_SIZE --kernel-trace -- python3 $BENCH --steps 1 --warmup 0 --respace-steps 2" \
    > gpurun_out/report_$TAG.log 2>&1 || { echo "report failed"; cat gpurun_out/report_$TAG.log; }
else
BUILD=$(python3 -c "import sys; sys.path.insert(0, 'diffusion-models-pytorch_amd'); import dmhip; print(dmhip.build_info())")
python3 tools/rocpd_report.py --tag $TAG --workload $WL --build "$BUILD" \
    --trace "$(find gpurun_out/prof_$TAG -name 'trace_results.db' | head -n 1)" > gpurun_out/report_$TAG.log 2>&1
fi
cat gpurun_out/report_$TAG.log
