#!/bin/bash
# isolate the ADM combined trajectory test across plan toggles and the previous build
cd "$(dirname "$0")/.." || exit 2
T=tests/test_gpu_adm.py::test_adm_combined_ddimcfg_trajectory
for cfg in "DM_AB_NONE=1" "DM_GN_NO_FIRST=1" "DM_GN_NO_UNITS=1" "DM_HIP_LIB=$PWD/tools/bin/libprev.so"; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python -m pytest -x -q $T --timeout 100 2>&1 | grep -E "passed|failed|AssertionError: step" | head -3
done
exit 0
