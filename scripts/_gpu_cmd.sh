set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_tgemm_gpu.py tests/test_engine_gpu.py -x -q -k "both_cores or engine or graph or prefix or hip_forward or tinyllama" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
MB_DECODE_B=1,8,64 MB_DECODE_C=512,2048 MB_KV_GB=8 MB_MAX_SEQS=64 timeout -k 10 300 python -u scripts/microbench.py --what decode > gpurun_out/decode_small.jsonl 2>&1
rc=$?; cat gpurun_out/decode_small.jsonl | grep bench; [ $rc -ne 0 ] && exit $rc
rm -f gpurun_out/harness/benchmark_results.csv gpurun_out/harness/benchmark_per_query.csv
bash scripts/harness_sweep.sh
