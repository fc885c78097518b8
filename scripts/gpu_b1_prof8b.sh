#!/bin/bash
# Per-kernel profile of the Llama-3-8B batch-1 decode step replay (C = 2048), plus the TP engine
# tests (the in-graph health vote path).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 MB_KV_GB=8 MB_MAX_SEQS=64 TMPDIR=/tmp
O=gpurun_out/b1p
mkdir -p $O
export DLLM_GEMM_PLANS=$O/plans.json
if [ -z "$SKIP_TP" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_tp_gpu.py tests/test_custom_ar_gpu.py -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $O/tp_tests.log 2>&1
  rc=$?; tail -2 $O/tp_tests.log; [ $rc -ne 0 ] && exit $rc
fi
# tune and cache the GEMM plans first, so the profiled run replays without autotune trials
MB_DECODE_B=1 MB_DECODE_C=2048 timeout -k 10 400 python3 scripts/microbench.py --what decode --model ${B1_MODEL:-llama-3-8b} \
  > $O/tune.log 2>&1 || exit $?
MB_DECODE_B=1 MB_DECODE_C=2048 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o l8b --output-format csv -- \
  python3 scripts/microbench.py --what decode --model ${B1_MODEL:-llama-3-8b} > $O/prof.log 2>&1 || exit $?
grep decode_step $O/prof.log | cut -c1-120
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python3 scripts/prof_summary.py "$f" 25 > $O/prof_summary.md && head -22 $O/prof_summary.md
find $O/prof -name '*kernel_trace.csv' -delete
