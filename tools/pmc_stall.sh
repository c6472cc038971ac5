#!/bin/bash
# Two SQ PMC passes (issue / wait / LDS / MFMA activity) over one conv microbenchmark shape and tile,
# summarised into gpurun_out/stall_<shape>_t<tile>.json (tools/pmc_summary.py).
#   SHAPE=res32_256 TILE=10 bash tools/pmc_stall.sh
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
S=${SHAPE:-res32_256}
T=${TILE:-0}
A="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
B="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
D=gpurun_out/stall_${S}_t${T}
timeout -s KILL 90 rocprofv3 --pmc $A --kernel-trace -d ${D}_a -o pmc -- \
    python3 tools/conv_bench.py --shape $S --math fp16x2 --iters 3 --tiles $T --ksplit ${KS:-0} > ${D}_a.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc $B --kernel-trace -d ${D}_b -o pmc -- \
    python3 tools/conv_bench.py --shape $S --math fp16x2 --iters 3 --tiles $T --ksplit ${KS:-0} > ${D}_b.log 2>&1 || exit $?
python3 tools/pmc_summary.py ${D}.json $(find ${D}_a ${D}_b -name '*.db') > ${D}.txt 2>&1
cat ${D}.txt
