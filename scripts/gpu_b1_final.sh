#!/bin/bash
# Single-stream decode step (batch 1, C = 2048), greedy and sampled (top-k 40, top-p 0.9, t = 0.8)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 MB_KV_GB=8 MB_MAX_SEQS=64 MB_DECODE_B=1 MB_DECODE_C=2048
O=gpurun_out/b1final
mkdir -p $O
for m in tinyllama-1.1b llama-3-8b; do
  for t in 0 0.8; do
    MB_TEMP=$t DLLM_GEMM_PLANS=$O/plans_$m.json timeout -k 10 300 python3 -u scripts/microbench.py --what decode \
      --model $m > $O/${m}_$t.log 2>&1 || exit $?
    echo "$m temp=$t"; grep decode_step $O/${m}_$t.log | cut -c1-110
  done
done
