set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_tgemm_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
MB_TUNE_SHAPES=2560x2048,2048x2048,11264x2048,2048x5632,32000x2048 MB_TUNE_M=128,256,320,384,512 \
  timeout -k 10 600 python -u scripts/microbench.py --what tune > gpurun_out/tune_tl.log 2>&1
rc=$?; grep "gemm M" gpurun_out/tune_tl.log | cut -c1-200; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --steps 4 --warmup 1 > gpurun_out/bench_deep.log 2>&1
rc=$?; grep '"metric"' gpurun_out/bench_deep.log; exit $rc
