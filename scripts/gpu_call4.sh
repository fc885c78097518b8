#!/bin/bash
# event-driven turn pipelining with the router on a side stream (driver's 20-step window)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
STEPS=20 WARMUP=5 bash scripts/ab_args.sh "--pipeline 2 --admit-every 8" "" "--pipeline 2 --admit-every 16" || exit $?
for i in 1 2 3; do tail -1 gpurun_out/ab/run$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], 'batch', d['avg_decode_batch'], 'p50', d['p50_latency_ms'], 'req', d['requests'])"; done
