#!/bin/bash
# Batch <= 8 decode GEMVs vs the streaming floor (scripts/exp/gemv_probe.py): default staging, then
# DLLM_GEMV_XG=1 (X carried in every W trip, batch 1-2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/gemv
PYTHONPATH=. timeout -k 10 300 python3 -u scripts/exp/gemv_probe.py 1 2 > gpurun_out/gemv/probe2.jsonl 2>&1 || exit $?
DLLM_GEMV_XG=1 PYTHONPATH=. timeout -k 10 300 python3 -u scripts/exp/gemv_probe.py 1 2 > gpurun_out/gemv/probe2_xg.jsonl 2>&1 || exit $?
echo gemvprobe ok
