#!/bin/bash
# BASELINE metric per strategy: the driver's bench window for each routing strategy, then the table.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/strat
for s in ${STRATS:-token heuristic semantic perf hybrid}; do
  timeout -k 10 330 python3 -u bench.py --gpus 1 --steps ${STEPS:-20} --warmup ${WARMUP:-5} --strategy $s \
    > gpurun_out/strat/$s.log 2>&1 || { echo "strategy $s rc=$?"; tail -5 gpurun_out/strat/$s.log; exit 1; }
  grep -o '"value": [0-9.]*' gpurun_out/strat/$s.log
done
python3 scripts/strategy_table.py gpurun_out/strat > gpurun_out/strat/table.md && cat gpurun_out/strat/table.md
