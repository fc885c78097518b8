#!/bin/bash
# Small-batch decode step: persistent work-list attention vs the static split grid (1x MI355X).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/svw
export DLLM_GEMM_PLANS=gpurun_out/svw/plans.json MB_KV_GB=8 MB_MAX_SEQS=64
export MB_DECODE_B=${MB_DECODE_B:-1,4,8,16,32} MB_DECODE_C=${MB_DECODE_C:-512,2048,8192} MB_MIN_CHUNKS=${MB_MIN_CHUNKS:-256,512}
for wl in 1 100000; do
  DLLM_ATTN_WL_MIN_BS=$wl timeout -k 10 300 python3 scripts/microbench.py --what decode \
    > gpurun_out/svw/wl$wl.log 2>&1 || { echo "wl=$wl failed"; tail -5 gpurun_out/svw/wl$wl.log; exit 1; }
  echo "wl_min_bs=$wl done"
done
