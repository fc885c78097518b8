#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
./scripts/gpu_wlab.sh || exit $?
STEPS=20 WARMUP=5 bash scripts/ab_args.sh "" "--groups 4" "--groups 8" "--groups 16"
