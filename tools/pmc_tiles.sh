#!/bin/bash
# SQ stall profile of one conv shape for several tiles (tools/pmc_stall.sh per tile + summary).
cd "$(dirname "$0")/.." || exit 2
for t in ${TILES:-0 7}; do
  rm -rf gpurun_out/stall_a gpurun_out/stall_b
  TILE=$t bash tools/pmc_stall.sh || exit $?
  python3 tools/pmc_summary.py gpurun_out/stall_${SHAPE:-res32_256}_t$t.json \
    $(find gpurun_out/stall_a gpurun_out/stall_b -name '*.db') || exit $?
done
