#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
STEPS=20 WARMUP=5 bash scripts/ab_args.sh "--gc-freeze 0" "" "--gc-freeze 0" "" || exit $?
for i in 1 2 3 4; do tail -1 gpurun_out/ab/run$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['gc_freeze'], d['value'], 'batch', d['avg_decode_batch'], 'p50', d['p50_latency_ms'])"; done
