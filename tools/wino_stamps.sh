#!/bin/bash
# Stamps of the Winograd kernel over several library builds: LIBS="a.so b.so" SHAPES="res32_128 res16_256"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
T=${T:-wino_st}
for lib in $LIBS; do
  for sh in ${SHAPES:-res32_128 res16_256}; do
    echo "== $lib"
    DM_HIP_LIB=$lib timeout -k 10 120 python3 tools/wino_stamps.py --shape $sh || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${T}.txt
