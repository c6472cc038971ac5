#!/bin/bash
# SQ stall profile of one conv shape for several tiles: tools/pmc_stall.sh per tile (it writes its own
# summary, gpurun_out/stall_<shape>_t<tile>.json).
cd "$(dirname "$0")/.." || exit 2
for t in ${TILES:-0 7}; do
  TILE=$t bash tools/pmc_stall.sh || exit $?
done
