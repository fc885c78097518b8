set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/microbench.py --what moe > gpurun_out/moe_bench.jsonl 2>&1
rc=$?; cat gpurun_out/moe_bench.jsonl | tail -14; exit $rc
