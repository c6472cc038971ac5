#!/bin/bash
# Round 5, first Winograd check: its unit tests + the CIFAR parity forwards, then a bench A/B against the direct conv.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_r5.py tests/test_gpu_parity.py -k "wino or small_map or forward_vs_reference" \
  -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_wino1_pytest.log 2>&1
rc=$?
tail -40 gpurun_out/r5_wino1_pytest.log
[ $rc -eq 0 ] || exit $rc
cp gpurun_out/parity_report.json gpurun_out/r5_wino1_parity.json 2>/dev/null
VAR=DM_CONV_WINO VAL=0 N=2 STEPS=4 bash tools/env_ab.sh 2>&1 | tee gpurun_out/r5_wino1_ab.txt
