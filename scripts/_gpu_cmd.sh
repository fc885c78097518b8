set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_tgemm_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
MB_TUNE_SHAPES=6144x4096,4096x4096,28672x4096,4096x14336,2560x2048,11264x2048 MB_TUNE_M=16,64,128,256 \
  timeout -k 10 600 python -u scripts/microbench.py --what tune > gpurun_out/tune_deep.log 2>&1
rc=$?; grep "gemm M" gpurun_out/tune_deep.log | cut -c1-250; exit $rc
