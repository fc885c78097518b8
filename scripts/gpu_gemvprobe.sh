#!/bin/bash
# GEMV numerics (fp32 references), then batch <= 8 decode GEMVs vs the streaming floor
# (scripts/exp/gemv_probe.py): default staging, then DLLM_GEMV_XG=1 (X carried in every W trip)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/gemv
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k gemv \
  tests/test_tgemm_gpu.py tests/test_kernels_gpu.py > gpurun_out/gemv/tests.log 2>&1 || { tail -30 gpurun_out/gemv/tests.log; exit 1; }
tail -2 gpurun_out/gemv/tests.log
DLLM_GEMV_XG=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k gemv \
  tests/test_tgemm_gpu.py tests/test_kernels_gpu.py > gpurun_out/gemv/tests_xg.log 2>&1 || { tail -30 gpurun_out/gemv/tests_xg.log; exit 1; }
tail -2 gpurun_out/gemv/tests_xg.log
PYTHONPATH=. timeout -k 10 300 python3 -u scripts/exp/gemv_probe.py 1 2 > gpurun_out/gemv/probe2.jsonl 2>&1 || exit $?
DLLM_GEMV_XG=1 PYTHONPATH=. timeout -k 10 300 python3 -u scripts/exp/gemv_probe.py 1 2 > gpurun_out/gemv/probe2_xg.jsonl 2>&1 || exit $?
echo gemvprobe ok
