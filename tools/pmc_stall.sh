#!/bin/bash
# Two SQ PMC passes (issue / wait / LDS / MFMA activity) over one conv microbenchmark shape.
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
S=${SHAPE:-res32_256}
A="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
B="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --pmc $A --kernel-trace -d gpurun_out/stall_a -o pmc -- \
    python3 tools/conv_bench.py --shape $S --math fp16x2 --iters 3 --tiles ${TILE:-0} > gpurun_out/stall_a.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc $B --kernel-trace -d gpurun_out/stall_b -o pmc -- \
    python3 tools/conv_bench.py --shape $S --math fp16x2 --iters 3 --tiles ${TILE:-0} > gpurun_out/stall_b.log 2>&1 || exit $?
echo done
