set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
: > gpurun_out/attnbench.jsonl
for cfg in "512 2048 0" "512 2048 1" "256 4096 1" "64 2048 1" "16 8192 0" "1 2048 0" "256 2048 1 32 8 128" "32 4096 1 32 8 128"; do
  timeout -k 10 120 ./scripts/exp/bin/attnbench $cfg >> gpurun_out/attnbench.jsonl 2>&1 || exit $?
done
cat gpurun_out/attnbench.jsonl
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "sample" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; exit $rc
