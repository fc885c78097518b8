#!/bin/bash
# Kernel numerics for the small-batch decode changes (GEMV 12-load trips, attention combine
# prefetch), then the single-stream decode step with the long-trip GEMV on / off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/b1ab
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_tgemm_gpu.py -k "gemv or paged_attention or fused_ops" \
  -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
export MB_KV_GB=8 MB_MAX_SEQS=64 DLLM_GEMM_PLANS=$O/plans.json
for v in ${LT:-1 0}; do
  DLLM_GEMV_LONG_TRIP=$v MB_DECODE_B=1,2 MB_DECODE_C=2048 timeout -k 10 300 python3 -u scripts/microbench.py --what decode \
    > $O/tiny_lt$v.log 2>&1 || exit $?
  echo "long_trip=$v"; grep decode_step $O/tiny_lt$v.log | cut -c1-110
done
for v in ${LT8:-1 0}; do
  DLLM_GEMV_LONG_TRIP=$v MB_DECODE_B=1 MB_DECODE_C=2048 timeout -k 10 300 python3 -u scripts/microbench.py --what decode --model llama-3-8b \
    > $O/l8b_lt$v.log 2>&1 || exit $?
  echo "8b long_trip=$v"; grep decode_step $O/l8b_lt$v.log | cut -c1-110
done
