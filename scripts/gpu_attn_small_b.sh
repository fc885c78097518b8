#!/bin/bash
# Decode step time at small batch vs the attention work-list chunking (split-K granularity) and the
# kernel's CH / block-table-prefetch variants (scripts/microbench.py decode, work list built).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/asb
export DLLM_GEMM_PLANS=gpurun_out/asb/plans.json MB_KV_GB=8 MB_MAX_SEQS=16
export MB_DECODE_B=${MB_DECODE_B:-1,8} MB_DECODE_C=${MB_DECODE_C:-512,2048,8192} MB_MIN_CHUNKS=${MB_MIN_CHUNKS:-64,128,256,512,1024,8192}
for v in "1 0" "2 0" "1 1" "2 1"; do
  set -- $v
  DLLM_ATTN_CH=$1 DLLM_ATTN_BT_PREFETCH=$2 timeout -k 10 300 python3 scripts/microbench.py --what decode \
    > gpurun_out/asb/ch$1_pf$2.log 2>&1 || { echo "ch=$1 pf=$2 failed"; tail -5 gpurun_out/asb/ch$1_pf$2.log; exit 1; }
  echo "ch=$1 pf=$2 done"
done
cat gpurun_out/asb/*.log | grep decode_step
