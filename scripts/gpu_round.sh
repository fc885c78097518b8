#!/bin/bash
# One round-check GPU session: every GPU test, smoke, the driver's bench command, then a rocprofv3
# kernel-stats profile of a short bench.  Each GPU step has its own time limit; the session stops at
# the first crash / abort / timeout (pytest rc 1 = test failures only, the rest still runs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/round
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
O=gpurun_out/round
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 720 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    -p no:cacheprovider > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -15 $O/pytest_gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -3 $O/smoke.log
  [ $rc -ne 0 ] && exit $rc
fi
export DLLM_GEMM_PLANS=$O/gemm_plans.json
timeout -k 10 400 python3 bench.py --gpus 1 --steps ${STEPS:-20} --warmup ${WARMUP:-5} ${BENCH_ARGS} > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 $O/bench.log
[ $rc -ne 0 ] && exit $rc
[ -n "$NO_PROF" ] && exit 0
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- \
  python3 bench.py --steps ${PSTEPS:-6} --warmup 1 ${BENCH_ARGS} > $O/prof_bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -1 $O/prof_bench.log
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python3 scripts/prof_summary.py "$f" 40 > $O/prof_summary.md && head -30 $O/prof_summary.md
find $O/prof -name "*trace*" -delete
exit $rc
