#!/bin/bash
# Fused-epilogue GEMV: numerics tests, engine tests, then the batch-1/8 decode replay profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_tgemm_gpu.py -k "gemv or fused_ops" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gemv_epi_tests.log 2>&1
rc=$?; tail -5 gpurun_out/gemv_epi_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/engine_tests.log 2>&1
rc=$?; tail -5 gpurun_out/engine_tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_decode_replay.sh
