#!/bin/bash
# GPU idle-gap analysis of the flagship bench (rocprofv3 kernel trace, no PMC)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/gaps
export TMPDIR=/tmp DLLM_GEMM_PLANS=gpurun_out/gaps/gemm_plans.json
timeout -k 10 400 python3 bench.py --steps 1 --warmup 0 ${BENCH_ARGS} > gpurun_out/gaps/tune.log 2>&1 || exit $?
timeout -k 10 ${PROF_TIMEOUT:-400} rocprofv3 --kernel-trace ${MEMCPY:+--memory-copy-trace} -d gpurun_out/gaps/prof -o bench --output-format csv -- \
  python3 bench.py --steps ${STEPS:-6} --warmup ${WARMUP:-2} ${BENCH_ARGS} > gpurun_out/gaps/bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -1 gpurun_out/gaps/bench.log | cut -c1-300
f=$(find gpurun_out/gaps/prof -name "*kernel_trace.csv" | head -1)
m=$(find gpurun_out/gaps/prof -name "*memory_copy_trace.csv" | head -1)
[ -n "$m" ] && f="$f,$m"
[ -n "$f" ] && python3 scripts/gap_summary.py "$f" 0.35 > gpurun_out/gaps/summary${TAG}.md && cat gpurun_out/gaps/summary${TAG}.md
find gpurun_out/gaps/prof -name "*.csv" -delete
exit $rc
