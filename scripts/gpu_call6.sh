#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=2 ./scripts/gpu_gaps.sh > /dev/null 2>&1 || exit $?
head -30 gpurun_out/gaps/summary2.md
mkdir -p gpurun_out/pgemm
PYTHONPATH=. timeout -k 10 600 python3 scripts/exp/prefill_gemm_probe.py 2048 8192 > gpurun_out/pgemm/probe_panel.jsonl 2>&1 || exit $?
echo call6 ok
