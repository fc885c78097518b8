#!/bin/bash
# Idle gaps and kernel split inside the driver's own window (20 steps after 5 warm-up steps)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
STEPS=20 WARMUP=5 PROF_TIMEOUT=700 TAG=${TAG:-_driver} ./scripts/gpu_gaps.sh
