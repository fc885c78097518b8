#!/bin/bash
# Driver-window GPU busy / idle: rocprofv3 kernel trace over the driver's own bench command, then
# scripts/gap_summary.py (first SKIP of the run dropped: start-up, tuning, warm-up).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
tag=${GAP_TAG:-gaps}
mkdir -p gpurun_out/$tag
timeout -k 10 900 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$tag/trace -o bench -- \
  python3 bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-5} ${BENCH_ARGS} > gpurun_out/$tag/bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; grep '^{"metric' gpurun_out/$tag/bench.log | cut -c1-300
f=$(find gpurun_out/$tag/trace -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python3 scripts/gap_summary.py "$f" ${SKIP:-0.35} > gpurun_out/$tag/gaps.md && head -40 gpurun_out/$tag/gaps.md
rm -rf gpurun_out/$tag/trace
exit $rc
