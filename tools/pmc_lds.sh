#!/bin/bash
# One SQ PMC pass (LDS bank conflicts, VALU / MFMA activity) over conv and GEMM microbenchmark shapes.
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
C="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS"
for s in ${SHAPES:-res32_256 qkv16}; do
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmc_lds_$s -o pmc -- \
      python3 tools/conv_bench.py --shape $s --math fp16x2 --iters 3 > gpurun_out/pmc_lds_$s.log 2>&1 || exit $?
done
timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmc_lds_gemm -o pmc -- \
    python3 tools/gemm_bench.py > gpurun_out/pmc_lds_gemm.log 2>&1 || exit $?
find gpurun_out -name "*counter_collection.csv" | head
