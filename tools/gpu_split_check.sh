cd /root/repo && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_split.py -x -q --timeout 120 --timeout-method thread > gpurun_out/split_tests.log 2>&1; rc=$?
tail -15 gpurun_out/split_tests.log
if [ $rc -ge 124 ] || [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python -u tools/conv_bench.py --iters 20 > gpurun_out/conv_bench_x3.log 2>&1; rc=$?
cat gpurun_out/conv_bench_x3.log | grep -v amdgpu.ids
exit $rc
