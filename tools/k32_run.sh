cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv_k32.py tests/test_gpu_conv_split.py -x -q --timeout 120 --timeout-method thread > gpurun_out/k32_tests.log 2>&1
rc=$?; tail -15 gpurun_out/k32_tests.log; [ $rc -ne 0 ] && exit $rc
for s in res32_128 res32_256 res32_384 res16_256; do
  timeout -k 10 120 python -u tools/conv_bench.py --shape $s --math fp16x2 --tiles 4,10,5,11 --iters 20 || exit $?
done
