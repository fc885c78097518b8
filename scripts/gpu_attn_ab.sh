#!/bin/bash
# Same-box A/B of decode-attention variants on the flagship bench (8 steps): default, CH=2, CH=2 + BT prefetch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/attn_ab
export DLLM_GEMM_PLANS=gpurun_out/attn_ab/plans.json
for v in "1 0" "2 0" "2 1" "1 0"; do
  set -- $v
  DLLM_ATTN_CH=$1 DLLM_ATTN_BT_PREFETCH=$2 timeout -k 10 400 python3 bench.py --steps ${STEPS:-8} --warmup 2 \
    > gpurun_out/attn_ab/ch$1_pf$2.log 2>&1 || { echo "ch=$1 pf=$2 failed"; tail -5 gpurun_out/attn_ab/ch$1_pf$2.log; exit 1; }
  echo "ch=$1 pf=$2: $(grep -o '"value": [0-9.]*' gpurun_out/attn_ab/ch$1_pf$2.log) $(grep -o '"t_decode_gpu_wait_s": [0-9.]*' gpurun_out/attn_ab/ch$1_pf$2.log)"
done
