#!/bin/bash
# Single-stream decode (the reference protocol's batch size): hipGraph step replay at B = 1-8 for
# TinyLlama and Llama-3-8B, then a per-kernel profile of the TinyLlama B = 1, C = 2048 replay.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 MB_KV_GB=8 MB_MAX_SEQS=64
O=gpurun_out/b1
mkdir -p $O
export DLLM_GEMM_PLANS=$O/plans.json
MB_DECODE_B=${B1_B:-1,2,4,8} MB_DECODE_C=${B1_C:-512,2048} timeout -k 10 300 python3 -u scripts/microbench.py --what decode \
  > $O/tiny.log 2>&1 || exit $?
grep decode_step $O/tiny.log | cut -c1-160
MB_DECODE_B=1 MB_DECODE_C=2048 timeout -k 10 300 python3 -u scripts/microbench.py --what decode --model llama-3-8b \
  > $O/l8b.log 2>&1 || exit $?
grep decode_step $O/l8b.log | cut -c1-160
[ -n "$NO_PROF" ] && exit 0
export TMPDIR=/tmp
MB_DECODE_B=1 MB_DECODE_C=2048 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o b1 --output-format csv -- \
  python3 scripts/microbench.py --what decode > $O/prof.log 2>&1 || exit $?
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python3 scripts/prof_summary.py "$f" 30 > $O/prof_summary.md && head -24 $O/prof_summary.md
