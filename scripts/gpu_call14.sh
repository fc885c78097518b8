#!/bin/bash
# SDMA copy engines vs blit kernels for the step loop's host copies (HSA_ENABLE_SDMA), driver window
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/ab14
mkdir -p $O
export DLLM_GEMM_PLANS=$O/gemm_plans.json
i=0
for sd in 0 1 0 1; do
  i=$((i+1))
  HSA_ENABLE_SDMA=$sd timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > $O/run$i.log 2>&1 \
    || { echo "run $i failed"; tail -20 $O/run$i.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/run$i.log').read().strip().splitlines()[-1]); print('sdma=$sd', d['value'], 'batch', d['avg_decode_batch'], 'p50', d['p50_latency_ms'], d['engine_time_split_s'])"
done
