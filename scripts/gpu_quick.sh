#!/bin/bash
# Targeted GPU check after a kernel change: the named test files (default: tgemm / flash / engine /
# models), then the driver's bench command.  Each step has its own time limit; stops at a crash.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/quick
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
TESTS=${TESTS:-"tests/test_tgemm_gpu.py tests/test_flash_gpu.py tests/test_engine_gpu.py tests/test_models_gpu.py"}
timeout -k 10 700 python -u -m pytest $TESTS -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
[ -n "$NO_BENCH" ] && exit 0
export DLLM_GEMM_PLANS=$O/gemm_plans.json
timeout -k 10 400 python3 bench.py --gpus 1 --steps ${STEPS:-20} --warmup ${WARMUP:-5} ${BENCH_ARGS} > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $O/bench.log | cut -c1-400
exit $rc
