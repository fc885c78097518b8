set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
MB_MOE_T=64 MB_MOE_PLAN_T=16,64,256,4096 timeout -k 10 600 python -u scripts/microbench.py --what moe > gpurun_out/moe_plans.jsonl 2>&1
rc=$?; cut -c1-330 gpurun_out/moe_plans.jsonl; exit $rc
