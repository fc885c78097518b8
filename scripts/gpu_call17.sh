#!/bin/bash
# Routing driver yielding to the engine's burst boundaries (--yield-to-engine), driver window A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/ab17
mkdir -p $O
export DLLM_GEMM_PLANS=$O/gemm_plans.json
i=0
for y in 1 0 1 0; do
  i=$((i+1))
  DLLM_SYNC_LOG=1 timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 --yield-to-engine $y > $O/run$i.log 2>&1 \
    || { echo "run $i failed"; tail -20 $O/run$i.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/run$i.log').read().strip().splitlines()[-1]); print('yield=$y', d['value'], 'batch', d['avg_decode_batch'], 'p50', d['p50_latency_ms'], d.get('step_loop_sync'))"
done
