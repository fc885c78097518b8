#!/bin/bash
# GIL switch interval A/B on the driver's window (engine step loop vs routing driver thread)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
STEPS=20 WARMUP=5 bash scripts/ab_args.sh "--gil-switch-ms 0.5" "--gil-switch-ms 5" "--gil-switch-ms 1" "--gil-switch-ms 0.5" || exit $?
