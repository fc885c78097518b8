#!/bin/bash
# GEMV numerics + probes, then the prefill/decode overlap probe
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
./scripts/gpu_gemvprobe.sh && ./scripts/gpu_overlap.sh
