#!/bin/bash
# scripts/exp/graph_gap_probe.py plain, then under a kernel trace + gap summary.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/ggap
timeout -k 10 300 python3 scripts/exp/graph_gap_probe.py > gpurun_out/ggap/plain.log 2>&1 || { tail -20 gpurun_out/ggap/plain.log; exit 1; }
tail -1 gpurun_out/ggap/plain.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ggap/trace -o p -- \
  python3 scripts/exp/graph_gap_probe.py > gpurun_out/ggap/traced.log 2>&1 || { tail -20 gpurun_out/ggap/traced.log; exit 1; }
tail -1 gpurun_out/ggap/traced.log
f=$(find gpurun_out/ggap/trace -name "*kernel_trace.csv" | head -1)
python3 scripts/gap_summary.py "$f" ${SKIP:-1.5} > gpurun_out/ggap/gaps.md && head -30 gpurun_out/ggap/gaps.md
rm -rf gpurun_out/ggap/trace
