set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_tgemm_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tgemm_gpu.log 2>&1
rc=$?; echo "tgemm rc=$rc"; tail -5 gpurun_out/tgemm_gpu.log; [ $rc -ne 0 ] && exit $rc
MB_TUNE_M=64,128,256,384,512 STEPS=6 bash scripts/gpu_perf_ab.sh
