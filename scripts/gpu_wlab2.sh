#!/bin/bash
# K-panel-major activations / weights in the decode-GEMM lab (M = 320 and 512)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/wlab
for M in 320 512; do
  timeout -k 10 300 ./labbin2/gemmlab $M 0 - notg > gpurun_out/wlab/panel_m$M.jsonl 2>&1 || exit $?
done
echo wlab2 ok
