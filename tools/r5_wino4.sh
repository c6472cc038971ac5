#!/bin/bash
# Winograd iteration 4: tests, conv bench main vs variant libs, stamps, bench A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
T=${T:-r5_w4}
timeout -k 10 300 python -u -m pytest tests/test_gpu_r5.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/${T}_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/${T}_pytest.log
[ $rc -eq 0 ] || exit $rc
for lib in "" $VARIANTS; do
  for sh in res32_128 res32_384 res16_256; do
    echo "lib=${lib:-main}"
    DM_HIP_LIB=$lib timeout -k 10 120 python3 tools/conv_bench.py --shape $sh --math fp16x2 --tiles 10,21 --iters 20 || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${T}_convbench.txt
for sh in res32_128 res16_256; do
  DM_HIP_LIB=tools/stampslib/libdm_stamps.so timeout -k 10 120 python3 tools/wino_stamps.py --shape $sh || exit 1
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${T}_stamps.txt
VAR=DM_CONV_WINO VAL=0 N=${N:-2} STEPS=4 bash tools/env_ab.sh 2>&1 | tee gpurun_out/${T}_ab.txt || exit 1
