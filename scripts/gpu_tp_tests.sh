#!/bin/bash
# Tensor-parallel GPU tests (N ranks on one GPU) + custom collectives + engine early-completion.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tp
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLLM_TEST_LOGDIR=gpurun_out/tp
timeout -k 10 900 python -u -m pytest tests/test_custom_ar_gpu.py tests/test_tp_gpu.py \
  "tests/test_engine_gpu.py::test_pipelined_short_request_completes_before_long_one" -x -v --timeout 600 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/tp/pytest.log 2>&1
rc=$?; echo "tp tests rc=$rc"; tail -30 gpurun_out/tp/pytest.log
exit $rc
