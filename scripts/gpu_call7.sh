#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
STEPS=20 WARMUP=5 bash scripts/ab_args.sh "" "--gil-switch-ms 0.5" "--gil-switch-ms 0.2" "--gil-switch-ms 1" || exit $?
for i in 1 2 3 4; do tail -1 gpurun_out/ab/run$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], 'batch', d['avg_decode_batch'], 'p50', d['p50_latency_ms'], 'req', d['requests'])"; done
