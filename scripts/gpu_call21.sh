#!/bin/bash
# A/B on one box: event driver blocking on the engines' completion queue (bench.py) vs the
# previous 1 ms poll over every in-flight ticket (scripts/exp/bench_poll_old.py = `git show
# a33ccc8:bench.py`, not kept in the tree), alternated.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/ab21
mkdir -p $O
export DLLM_GEMM_PLANS=$O/gemm_plans.json DLLM_THREAD_CPU=1
i=0
for b in bench.py scripts/exp/bench_poll_old.py bench.py scripts/exp/bench_poll_old.py; do
  i=$((i+1))
  PYTHONPATH=. timeout -k 10 600 python3 $b --steps 20 --warmup 5 > $O/run$i.log 2>&1 \
    || { echo "run $i failed"; tail -30 $O/run$i.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('$O/run$i.log').read().strip().splitlines()[-1])
print('$b', d['value'], d['p50_latency_ms'], d.get('thread_cpu_share'))"
done
