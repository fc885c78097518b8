#!/bin/bash
# Split-vocab sampler (small batches): sampler tests, then the batch-1 / 2 / 8 decode step with the
# split on / off / on (DLLM_SAMPLE_SPLIT_MAX_B=0 disables it), greedy and sampled rows.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/ssplit
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_tp_sampler.py -k "sampl" \
  -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
export MB_KV_GB=8 MB_MAX_SEQS=64
i=0
for mx in 8 0 8; do
  i=$((i+1))
  for t in 0 0.8; do
    DLLM_SAMPLE_SPLIT_MAX_B=$mx MB_TEMP=$t DLLM_GEMM_PLANS=$O/plans_t.json MB_DECODE_B=1,2,8 MB_DECODE_C=2048 \
      timeout -k 10 300 python3 -u scripts/microbench.py --what decode > $O/tiny_${i}_$t.log 2>&1 || exit $?
    echo "split_max_b=$mx temp=$t"; grep decode_step $O/tiny_${i}_$t.log | cut -c1-110
  done
done
DLLM_SAMPLE_SPLIT_MAX_B=8 MB_TEMP=0.8 DLLM_GEMM_PLANS=$O/plans_8.json MB_DECODE_B=1 MB_DECODE_C=2048 timeout -k 10 300 \
  python3 -u scripts/microbench.py --what decode --model llama-3-8b > $O/l8b_on.log 2>&1 || exit $?
echo "8b split on"; grep decode_step $O/l8b_on.log | cut -c1-110
DLLM_SAMPLE_SPLIT_MAX_B=0 MB_TEMP=0.8 DLLM_GEMM_PLANS=$O/plans_8.json MB_DECODE_B=1 MB_DECODE_C=2048 timeout -k 10 300 \
  python3 -u scripts/microbench.py --what decode --model llama-3-8b > $O/l8b_off.log 2>&1 || exit $?
echo "8b split off"; grep decode_step $O/l8b_off.log | cut -c1-110
