#!/bin/bash
# Host cost of launching one admission prefill chunk (scripts/exp/prefill_host_probe.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/pfhost
PYTHONPATH=. timeout -k 10 400 python3 -u scripts/exp/prefill_host_probe.py > gpurun_out/pfhost/probe.log 2>&1 || { tail -30 gpurun_out/pfhost/probe.log; exit 1; }
head -60 gpurun_out/pfhost/probe.log
