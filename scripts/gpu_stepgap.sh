#!/bin/bash
# Kernel-trace of back-to-back decode-graph replays (scripts/exp/step_copy_probe.py): idle between steps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out/stepgap
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/stepgap/prof -o sg --output-format csv -- \
  python3 scripts/exp/step_copy_probe.py > gpurun_out/stepgap/probe.log 2>&1 || { tail -20 gpurun_out/stepgap/probe.log; exit 1; }
f=$(find gpurun_out/stepgap/prof -name "*kernel_trace.csv" | head -1)
python3 scripts/gap_summary.py "$f" 1.5 > gpurun_out/stepgap/summary.md
find gpurun_out/stepgap/prof -name "*.csv" -delete
head -12 gpurun_out/stepgap/summary.md; grep -n "idle ms" -A10 gpurun_out/stepgap/summary.md
