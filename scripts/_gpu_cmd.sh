set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_tgemm_gpu.py -x -q -k "both_cores" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/microbench.py --what post,flash > gpurun_out/post_flash.jsonl 2>&1
rc=$?; cat gpurun_out/post_flash.jsonl; exit $rc
