#!/bin/bash
# A/B the flagship bench under two env settings, alternating (ABAB) in one GPU session.
#   A="DLLM_DECODE_SORT=0" B="DLLM_DECODE_SORT=1" STEPS=8 bash scripts/ab_bench.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
STEPS=${STEPS:-8}
export DLLM_GEMM_PLANS=gpurun_out/ab/gemm_plans.json
for round in 1 2; do
  for v in A B; do
    eval "envs=\${$v}"
    env $envs timeout -k 10 600 python3 bench.py --steps $STEPS --warmup 2 > gpurun_out/ab/$v$round.log 2>&1 || exit $?
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab/$v$round.log').read().strip().splitlines()[-1]); print('$v$round', '$envs', d['value'], d['engine_time_split_s'])"
  done
done
