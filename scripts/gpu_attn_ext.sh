#!/bin/bash
# Extended decode work list: attention numerics, engine tests, small-batch decode steps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/ae
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_decode_attn_gpu.py -k "attention or decode" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ae/tests.log 2>&1
rc=$?; tail -3 gpurun_out/ae/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ae/engine.log 2>&1
rc=$?; tail -3 gpurun_out/ae/engine.log; [ $rc -ne 0 ] && exit $rc
export DLLM_GEMM_PLANS=gpurun_out/ae/plans.json MB_KV_GB=8 MB_MAX_SEQS=64
MB_DECODE_B=${MB_DECODE_B:-1,2,8,32} MB_DECODE_C=${MB_DECODE_C:-512,2048,8192} timeout -k 10 300 python3 scripts/microbench.py --what decode > gpurun_out/ae/decode.log 2>&1
rc=$?; grep decode_step gpurun_out/ae/decode.log | cut -c1-110; exit $rc
