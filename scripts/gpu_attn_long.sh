#!/bin/bash
# Decode attention scheduling at the driver window's long contexts (B = 496, C = 2048 / 4096):
# persistent grid size x work items per workgroup, whole decode step (scripts/microbench.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 MB_KV_GB=64 MB_MAX_SEQS=512
O=gpurun_out/attnlong
mkdir -p $O
export DLLM_GEMM_PLANS=$O/plans.json
for cfg in "512 1" "1024 1" "512 2" "2048 1" "1024 2" "256 1"; do
  set -- $cfg
  DLLM_ATTN_PGRID=$1 DLLM_ATTN_ITEMS_PER_WG=$2 MB_DECODE_B=496 MB_DECODE_C=2048,4096 timeout -k 10 300 \
    python3 -u scripts/microbench.py --what decode > $O/g$1_i$2.log 2>&1 || { tail -20 $O/g$1_i$2.log; exit 1; }
  echo "pgrid=$1 items=$2"; grep decode_step $O/g$1_i$2.log | cut -c1-120
done
