#!/bin/bash
# Flagship bench: barrier-per-turn vs conversation groups (turn pipelining), one box, plans cached.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/groups
export DLLM_GEMM_PLANS=gpurun_out/groups/gemm_plans.json
STEPS=${STEPS:-8}
for g in 1 4 2 1; do
  timeout -k 10 600 python3 bench.py --steps $STEPS --warmup 2 --groups $g > gpurun_out/groups/g$g.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/groups/g$g.log').read().strip().splitlines()[-1]); print('groups=$g', d['value'], d['p50_latency_ms'], d['avg_decode_batch'], d['engine_time_split_s'])"
done
