#!/bin/bash
# Single-stream decode step (TinyLlama, B = 1 / 4, C = 2048) across the decode-attention runtime
# knobs: workgroup waves, shortest work unit, chunks per trip, block-table prefetch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 MB_KV_GB=8 MB_MAX_SEQS=64
O=gpurun_out/attn_b1
mkdir -p $O
export DLLM_GEMM_PLANS=$O/plans.json MB_DECODE_B=1,4 MB_DECODE_C=2048 MB_MIN_CHUNKS=128,256,512,1024
for v in "" "DLLM_ATTN_WAVES=4" "DLLM_ATTN_CH=2" "DLLM_ATTN_BT_PREFETCH=1" "DLLM_ATTN_CH=2 DLLM_ATTN_BT_PREFETCH=1"; do
  tag=$(echo "base $v" | tr ' =' '__')
  env $v timeout -k 10 300 python3 -u scripts/microbench.py --what decode > $O/$tag.log 2>&1 || exit $?
  echo "== $v"; grep decode_step $O/$tag.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['B'], d['C'], 'min_chunk', d['min_chunk'], d['ms'])"
done
