#!/bin/bash
# Batch-1 decode step vs the shortest attention work unit, for head dims 64 / 96 / 128
# (TinyLlama, phi3-mini, Llama-3-8B), C = 2048.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 MB_KV_GB=8 MB_MAX_SEQS=64 MB_DECODE_B=1,4 MB_DECODE_C=2048 MB_MIN_CHUNKS=64,128,256,512
O=gpurun_out/attn_chunk
mkdir -p $O
for m in ${MODELS:-llama-3-8b phi3-mini tinyllama-1.1b}; do
  DLLM_GEMM_PLANS=$O/plans_$m.json timeout -k 10 300 python3 -u scripts/microbench.py --what decode --model $m > $O/$m.log 2>&1 || exit $?
  echo "== $m"; grep decode_step $O/$m.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['B'], d['C'], 'min_chunk', d['min_chunk'], d['ms'])"
done
