#!/bin/bash
# Two SQ PMC passes over a short C3 bench run (2 denoising steps), summarised per kernel into
# gpurun_out/pmc_c3.json / .txt (tools/pmc_summary.py); GREP selects the kernels printed.
#   GREP='attn_block|linear_k32' bash tools/pmc_c3.sh
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
A="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
B="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
D=gpurun_out/pmc_c3
CMD="python3 bench.py --steps 1 --warmup 0 --respace-steps 2 --no-cpu-baseline --no-profile ${ARGS}"
timeout -s KILL 120 rocprofv3 --pmc $A --kernel-trace -d ${D}_a -o pmc -- $CMD > ${D}_a.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc $B --kernel-trace -d ${D}_b -o pmc -- $CMD > ${D}_b.log 2>&1 || exit $?
python3 tools/pmc_summary.py ${D}.json $(find ${D}_a ${D}_b -name '*.db') > ${D}.txt 2>&1
grep -E -A20 "${GREP:-attn_block}" ${D}.txt
