#!/bin/bash
# Flagship bench at several concurrency levels (conversations per GPU), one box: throughput vs p50.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/conc
export DLLM_GEMM_PLANS=gpurun_out/conc/plans.json
for c in ${CONVS_LIST:-256 512 768 1024}; do
  kv=$(( c <= 512 ? 64 : 128 ))
  timeout -k 10 500 python3 bench.py --steps 8 --warmup 2 --convs $c --kv-gb $kv > gpurun_out/conc/c$c.log 2>&1 || { echo "convs=$c failed"; tail -5 gpurun_out/conc/c$c.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/conc/c$c.log').read().strip().splitlines()[-1]); print($c, d['value'], d['p50_latency_ms'], d['p90_latency_ms'], d['avg_decode_batch'])"
done
