#!/bin/bash
# Batch-1 GEMV with X carried in every weight trip (DLLM_GEMV_XG, default on at batch 1) vs the LDS
# stage: GEMV numerics, then the single-stream decode step (TinyLlama, Llama-3-8B), XG 1 / 0 / 1
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/b1xg
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_tgemm_gpu.py -k "gemv or fused_ops or embedding" \
  -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
export MB_KV_GB=8 MB_MAX_SEQS=64
i=0
for v in 1 0 1; do
  i=$((i+1))
  DLLM_GEMV_XG=$v DLLM_GEMM_PLANS=$O/plans_t$i.json MB_DECODE_B=1,2 MB_DECODE_C=2048 timeout -k 10 300 \
    python3 -u scripts/microbench.py --what decode > $O/tiny_$i.log 2>&1 || exit $?
  echo "xg=$v"; grep decode_step $O/tiny_$i.log | cut -c1-110
  DLLM_GEMV_XG=$v DLLM_GEMM_PLANS=$O/plans_8_$i.json MB_DECODE_B=1 MB_DECODE_C=2048 timeout -k 10 300 \
    python3 -u scripts/microbench.py --what decode --model llama-3-8b > $O/l8b_$i.log 2>&1 || exit $?
  echo "8b xg=$v"; grep decode_step $O/l8b_$i.log | cut -c1-110
done
