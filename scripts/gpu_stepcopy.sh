#!/bin/bash
# Cost of the decode step's host copies on the GPU timeline (scripts/exp/step_copy_probe.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/stepcopy
PYTHONPATH=. timeout -k 10 400 python3 -u scripts/exp/step_copy_probe.py > gpurun_out/stepcopy/probe.jsonl 2> gpurun_out/stepcopy/err.log \
  || { tail -20 gpurun_out/stepcopy/err.log; exit 1; }
PROBE_C=4000 PYTHONPATH=. timeout -k 10 400 python3 -u scripts/exp/step_copy_probe.py >> gpurun_out/stepcopy/probe.jsonl 2>> gpurun_out/stepcopy/err.log \
  || { tail -20 gpurun_out/stepcopy/err.log; exit 1; }
cat gpurun_out/stepcopy/probe.jsonl
