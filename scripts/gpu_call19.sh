#!/bin/bash
# Admission cadence with in-burst joins: --admit-every 4 / 8 / 16 / 4, driver window
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/ab19
mkdir -p $O
export DLLM_GEMM_PLANS=$O/gemm_plans.json
i=0
for ae in ${AES:-4 8 16 2}; do
  i=$((i+1))
  timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 --admit-every $ae > $O/run$i.log 2>&1 \
    || { echo "run $i failed"; tail -30 $O/run$i.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/run$i.log').read().strip().splitlines()[-1]); print('admit_every=$ae', d['value'], 'batch', d['avg_decode_batch'], 'p50', d['p50_latency_ms'], 'ttft', d.get('ttft_ms_p50'), d['engine_time_split_s']['t_prefill_s'])"
done
