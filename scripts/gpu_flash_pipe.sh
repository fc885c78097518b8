#!/bin/bash
# Flash prefill: numerics of the pipelined P.V variant (DLLM_FLASH_PIPE=1), then TFLOP/s of both
# variants (scripts/microbench.py --what flash: cold causal prefill, 1k-16k tokens, d 64 / 128 / 96).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/flashpipe
mkdir -p $O
DLLM_FLASH_PIPE=1 timeout -k 10 600 python -u -m pytest tests/test_flash_gpu.py -x -q --timeout 200 --timeout-method thread \
  -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for v in 0 1; do
  DLLM_FLASH_PIPE=$v timeout -k 10 400 python3 -u scripts/microbench.py --what flash > $O/bench_pipe$v.log 2>&1 || exit $?
  echo "== pipe=$v"; grep flash_prefill $O/bench_pipe$v.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['B'], d['L'], d['nq'], d['nkv'], d['d'], d['flash_us'], d['flash_TFLOPs'])"
done
