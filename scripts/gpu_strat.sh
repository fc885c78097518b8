#!/bin/bash
# per-strategy flagship runs on the round-4 tree (driver's window: 20 timed steps after 5 warm-up)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
STEPS=20 WARMUP=5 STRATEGIES="${STRATEGIES:-token heuristic semantic perf hybrid}" bash scripts/strategy_sweep.sh || exit $?
python3 scripts/strategy_table.py
