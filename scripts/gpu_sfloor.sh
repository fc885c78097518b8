#!/bin/bash
# Streaming-read floor for decode weight matrices (scripts/exp/streamfloor.hip)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sfloor
timeout -k 10 300 ./labbin2/streamfloor > gpurun_out/sfloor/streamfloor.jsonl 2>&1 || exit $?
echo sfloor ok
