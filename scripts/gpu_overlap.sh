#!/bin/bash
# Prefill chunk on a side stream vs decode-step replays (scripts/exp/prefill_overlap_probe.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/overlap
for K in 4 8; do
  PROBE_K=$K PYTHONPATH=. timeout -k 10 400 python3 -u scripts/exp/prefill_overlap_probe.py \
    >> gpurun_out/overlap/probe.jsonl 2> gpurun_out/overlap/err_$K.log || { tail -20 gpurun_out/overlap/err_$K.log; exit 1; }
done
cat gpurun_out/overlap/probe.jsonl
