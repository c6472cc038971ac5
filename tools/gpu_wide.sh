cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_r6.py tests/test_gpu_r5.py -x -q --timeout 300 --timeout-method thread > gpurun_out/wide_pytest.log 2>&1 || { tail -60 gpurun_out/wide_pytest.log; exit 1; }
tail -3 gpurun_out/wide_pytest.log
N=1 ARGS="--workload c4 --respace-steps 5" bash tools/ab_bench.sh
