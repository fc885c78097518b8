#!/bin/bash
# Flagship bench once per routing strategy (BASELINE metric: routed p50 latency + tok/s per
# strategy).  One GPU session, sequential, stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/strat
export DLLM_GEMM_PLANS=gpurun_out/strat/gemm_plans.json
STEPS=${STEPS:-8}; WARMUP=${WARMUP:-2}
for s in ${STRATEGIES:-token heuristic semantic perf hybrid}; do
  timeout -k 10 600 python3 bench.py --steps $STEPS --warmup $WARMUP --strategy $s ${BENCH_ARGS} > gpurun_out/strat/$s.log 2>&1 || { echo "$s failed rc=$?"; tail -20 gpurun_out/strat/$s.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/strat/$s.log').read().strip().splitlines()[-1]); print('$s', d['value'], 'p50', d['p50_latency_ms'], 'small', d['small_tier_share'])"
done
