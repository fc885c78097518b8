#!/bin/bash
# Fused-op numerics + engine tests, then the small-batch decode step (attention work list built).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/sb
timeout -k 10 600 python -u -m pytest tests/test_tgemm_gpu.py -k "gemv or fused_ops or swiglu or qkv" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/sb/tests.log 2>&1
rc=$?; tail -3 gpurun_out/sb/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/sb/engine.log 2>&1
rc=$?; tail -3 gpurun_out/sb/engine.log; [ $rc -ne 0 ] && exit $rc
export DLLM_GEMM_PLANS=gpurun_out/sb/plans.json MB_KV_GB=8 MB_MAX_SEQS=64 DLLM_VERBOSE=1
MB_DECODE_B=${MB_DECODE_B:-1,2,4,8,16,32} MB_DECODE_C=${MB_DECODE_C:-512,2048} timeout -k 10 300 python3 scripts/microbench.py --what decode > gpurun_out/sb/decode.log 2>&1
rc=$?; grep decode_step gpurun_out/sb/decode.log | cut -c1-120; exit $rc
