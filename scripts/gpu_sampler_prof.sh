#!/bin/bash
# Kernel times of the batch-1 sampled decode step with the split-vocab sampler on / off (rocprofv3).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
O=gpurun_out/ssprof
mkdir -p $O
export MB_KV_GB=8 MB_MAX_SEQS=64 MB_TEMP=0.8 MB_DECODE_B=1 MB_DECODE_C=2048
for m in llama-3-8b tinyllama-1.1b; do
  for mx in 8 0; do
    DLLM_SAMPLE_SPLIT_MAX_B=$mx DLLM_GEMM_PLANS=$O/plans_$m.json timeout -k 10 300 rocprofv3 --kernel-trace --stats \
      -d $O/p_${m}_$mx -o run --output-format csv -- python3 -u scripts/microbench.py --what decode --model $m \
      > $O/run_${m}_$mx.log 2>&1 || exit $?
    f=$(find $O/p_${m}_$mx -name "*kernel_stats.csv" | head -1)
    echo "$m split_max_b=$mx"; grep decode_step $O/run_${m}_$mx.log | cut -c1-100
    grep -i "sample" "$f" | cut -c1-200
    find $O/p_${m}_$mx -name "*trace*" -delete
  done
done
