#!/bin/bash
# One decode-graph replay of MODEL at batch B, context C under rocprofv3 (kernel table of the last replay).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
M=${MODEL:-phi3-mini}; B=${B:-1}; C=${C:-1024}
d=gpurun_out/rp_${M}_b${B}; mkdir -p $d
export DLLM_GEMM_PLANS=$d/plans.json MB_KV_GB=${KV:-16} MB_MAX_SEQS=16 MB_DECODE_B=$B MB_DECODE_C=$C
timeout -k 10 300 python3 scripts/microbench.py --model $M --what decode > $d/tune.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace -d $d -o rp --output-format csv -- python3 scripts/microbench.py --model $M --what decode > $d/run.log 2>&1 || exit $?
f=$(find $d -name "*kernel_trace.csv" | head -1); python3 scripts/replay_trace.py "$f" > $d/replay.md; rm -f "$f"
grep decode_step $d/tune.log | cut -c1-150; head -20 $d/replay.md
