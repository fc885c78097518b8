#!/bin/bash
# Multi-process and harness validation on one GPU: the pools-topology rehearsal test (2 / 4 ranks vs a
# single-process run), the tensor-parallel engine tests, then the reference-model legacy harness
# (phi3-mini + Llama-3-8B, energy per query from the GPU energy counter).  Each step has its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/validate
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLLM_TEST_LOGDIR=$O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest ${TESTS:-tests/test_pools_gpu.py tests/test_tp_gpu.py} -m gpu -x -v -s \
    --timeout 900 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|agreement|passed|failed" $O/pytest.log | tail -12
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
[ -n "$NO_HARNESS" ] && exit 0
export DLLM_GEMM_PLANS=$O/gemm_plans_ref.json
timeout -k 10 900 python3 -u scripts/legacy_ref_models.py $O/legacy_ref > $O/legacy_ref.log 2>&1
rc=$?; echo "legacy harness rc=$rc"; tail -8 $O/legacy_ref.log | cut -c1-300
exit $rc
