#!/bin/bash
# SQ counters of the Winograd kernel on one conv shape, HEAD build (tools/lib/libprev.so) and working tree:
#   SHAPE=res32_128 bash tools/pmc_wino.sh   -> gpurun_out/pmc_wino_{prev,new}.txt
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
SHAPE=${SHAPE:-res32_128}
A="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
B="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE"
for v in ${VARIANTS:-prev new}; do
  if [ "$v" = prev ]; then export DM_HIP_LIB=$PWD/tools/lib/libprev.so; else unset DM_HIP_LIB; fi
  D=gpurun_out/pmc_wino_${v}
  rm -rf ${D}_a ${D}_b
  CMD="python3 tools/conv_bench.py --shape $SHAPE --math fp16x2 --tiles 21 --iters 5"
  timeout -s KILL 90 rocprofv3 --pmc $A --kernel-trace -d ${D}_a -o pmc -- $CMD > ${D}_a.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc $B --kernel-trace -d ${D}_b -o pmc -- $CMD > ${D}_b.log 2>&1 || exit $?
  python3 tools/pmc_summary.py ${D}.json $(find ${D}_a ${D}_b -name '*.db') > ${D}.txt 2>&1
  echo "== $v $SHAPE"; grep -A20 conv_wino ${D}.txt
  rm -rf ${D}_a ${D}_b
done
