#!/bin/bash
# Kernel-level profile of the flagship bench (rocprofv3 kernel trace + stats, no PMC).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/${PROF_TAG:-prof}
export TMPDIR=/tmp
STEPS=${STEPS:-3}
# first a plain run that autotunes and saves the GEMM plans, so the profiled run below does not
# include the tuning sweeps (its kernel statistics then cover warm-up + timed steps only)
export DLLM_GEMM_PLANS=gpurun_out/${PROF_TAG:-prof}/gemm_plans.json
timeout -k 10 600 python3 bench.py --steps 1 --warmup 0 ${BENCH_ARGS} > gpurun_out/${PROF_TAG:-prof}_tune.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${PROF_TAG:-prof} -o bench --output-format csv -- \
  python3 bench.py --steps $STEPS --warmup 1 ${BENCH_ARGS} > gpurun_out/${PROF_TAG:-prof}_bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/${PROF_TAG:-prof}_bench.log
f=$(find gpurun_out/${PROF_TAG:-prof} -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python3 scripts/prof_summary.py "$f" 40 > gpurun_out/${PROF_TAG:-prof}/summary.md && head -50 gpurun_out/${PROF_TAG:-prof}/summary.md
find gpurun_out/${PROF_TAG:-prof} -name "*trace*" -delete
exit $rc
