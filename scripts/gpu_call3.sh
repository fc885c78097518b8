#!/bin/bash
# event-driven turn pipelining A/B (driver's 20-step window) + prefill GEMM probe
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pgemm
STEPS=20 WARMUP=5 bash scripts/ab_args.sh "" "--pipeline 2 --admit-every 8" "--pipeline 2 --admit-every 16" "--pipeline 2 --admit-every 4" || exit $?
timeout -k 10 600 python3 scripts/exp/prefill_gemm_probe.py 2048 4096 8192 > gpurun_out/pgemm/probe.jsonl 2>&1 || exit $?
echo call3 ok
