#!/bin/bash
# Sampler numerics, then its cost per logit distribution (scripts/exp/sampler_probe.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/sprobe2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_tp_sampler.py tests/test_tensor_parallel.py -k "sampl" \
  -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
DLLM_AUTOTUNE=0 timeout -k 10 400 python3 -u scripts/exp/sampler_probe.py > $O/out.log 2>&1
rc=$?; grep "{" $O/out.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 ./expbin/sampler_phases > $O/phases.jsonl 2>&1; rc=$?; cat $O/phases.jsonl; exit $rc
