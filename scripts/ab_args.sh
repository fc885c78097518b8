#!/bin/bash
# Run the flagship bench once per argument set (one GPU session, sequential, stop on failure).
#   bash scripts/ab_args.sh "--pipeline 0" "--pipeline 1" "--pipeline 1 --convs 512"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
export DLLM_GEMM_PLANS=gpurun_out/ab/gemm_plans.json
STEPS=${STEPS:-4}; WARMUP=${WARMUP:-1}
i=0
for args in "$@"; do
  i=$((i+1))
  timeout -k 10 600 python3 bench.py --steps $STEPS --warmup $WARMUP $args > gpurun_out/ab/run$i.log 2>&1 || { echo "run $i ($args) failed rc=$?"; tail -20 gpurun_out/ab/run$i.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab/run$i.log').read().strip().splitlines()[-1]); print('run$i', '$args', d['value'], 'p50', d['p50_latency_ms'], d['engine_time_split_s'])"
done
