#!/bin/bash
# Fused GEMM numerics, then the engine / model-family tests that run through it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_tgemm_gpu.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/tgemm_gpu.log 2>&1
rc=$?; echo "tgemm rc=$rc"; tail -25 gpurun_out/tgemm_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests/test_models_gpu.py tests/test_engine_gpu.py -x -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/models_gpu.log 2>&1
rc=$?; echo "models rc=$rc"; tail -25 gpurun_out/models_gpu.log
exit $rc
