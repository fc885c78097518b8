#!/bin/bash
# Step-loop diagnostics on the driver's window: per-step host prep and wait for the in-flight step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/ab16
mkdir -p $O
export DLLM_GEMM_PLANS=$O/gemm_plans.json
DLLM_SYNC_LOG=1 timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > $O/run1.log 2>&1 || { tail -20 $O/run1.log; exit 1; }
python3 -c "import json; d=json.loads(open('$O/run1.log').read().strip().splitlines()[-1]); print(d['value'], d['step_loop_sync'], d['engine_time_split_s'])"
