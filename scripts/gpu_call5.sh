#!/bin/bash
# GPU test suite (new TP vote-fault / fused-SP / EP-graph / config-5 / failover tests), admission
# cadence A/B for the event-driven driver, prefill GEMM probe
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/t gpurun_out/pgemm
timeout -k 10 900 python -u -m pytest tests/test_tp_gpu.py tests/test_pools_gpu.py -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/t/tp_pools.log 2>&1
rc=$?; tail -15 gpurun_out/t/tp_pools.log; [ $rc -ne 0 ] && exit $rc
STEPS=20 WARMUP=5 bash scripts/ab_args.sh "--pipeline 2 --admit-every 32" "--pipeline 2 --admit-every 64" || exit $?
PYTHONPATH=. timeout -k 10 600 python3 scripts/exp/prefill_gemm_probe.py 2048 4096 8192 > gpurun_out/pgemm/probe.jsonl 2>&1 || exit $?
echo call5 ok
