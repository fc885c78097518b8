#!/bin/bash
# GEMM autotune table (TinyLlama shapes) + flagship bench A/B: fused layer vs unfused (same box).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ "${SKIP_TUNE:-0}" != "1" ]; then
MB_TUNE_SHAPES=${MB_TUNE_SHAPES:-2560x2048,2048x2048,11264x2048,2048x5632,32000x2048} \
  timeout -k 10 600 python -u scripts/microbench.py --what tune > gpurun_out/tune.log 2>&1
rc=$?; echo "tune rc=$rc"; grep "best=" gpurun_out/tune.log | tail -45
if [ $rc -ne 0 ]; then exit $rc; fi
fi
for f in ${FUSED_LIST:-1 0}; do
  DLLM_FUSED=$f DLLM_GEMM_PLANS=gpurun_out/plans_$f.json timeout -k 10 900 python -u bench.py --steps ${STEPS:-4} --warmup 1 \
    > gpurun_out/bench_fused$f.log 2>&1
  rc=$?; echo "bench fused=$f rc=$rc"; tail -2 gpurun_out/bench_fused$f.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
