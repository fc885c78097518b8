#!/bin/bash
# Per-model routed bench line + rocprof kernel table on one MI355X:
#   MODEL=llama-3-8b CONVS=128 STEPS=2 bash scripts/gpu/model_bench.sh
# Run 1 tunes the GEMM plans (saved); run 2 is the profiled one (kernel trace + stats, no PMC).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
M=${MODEL:?MODEL}
CONVS=${CONVS:-128}
STEPS=${STEPS:-2}
LIMIT=${LIMIT:-540}
out=gpurun_out/model_$M
mkdir -p $out
export DLLM_GEMM_PLANS=$out/gemm_plans.json
ARGS="--model $M --convs $CONVS --steps $STEPS --warmup 1 --kv-gb ${KV_GB:-48} ${BENCH_ARGS}"
timeout -k 10 $LIMIT python3 -u bench.py $ARGS > $out/bench.log 2>&1
rc=$?; echo "bench $M rc=$rc"; grep '"metric"' $out/bench.log || tail -20 $out/bench.log
[ $rc -ne 0 ] && exit $rc
[ "${PROFILE:-1}" = "1" ] || exit 0
timeout -k 10 $LIMIT rocprofv3 --kernel-trace --stats -d $out/prof -o bench --output-format csv -- \
  python3 bench.py $ARGS > $out/prof_bench.log 2>&1
rc=$?; echo "rocprof $M rc=$rc"
f=$(find $out/prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python3 scripts/prof_summary.py "$f" 40 > $out/summary.md && head -30 $out/summary.md
find $out/prof -name "*trace*" -delete
exit $rc
