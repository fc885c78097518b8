#!/bin/bash
# Split-KV flash prefill: numerics (all flash tests), then one prompt's new tokens behind a long
# cached history with the split auto-chosen vs off (scripts/microbench.py --what flash_cached)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/flashsplit
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_flash_gpu.py -x -q --timeout 200 --timeout-method thread \
  -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED|Mismatch" $O/tests.log | head -20; exit $rc; }
timeout -k 10 400 python3 -u scripts/microbench.py --what flash_cached > $O/cached.log 2>&1 || { tail -20 $O/cached.log; exit 1; }
grep flash_cached $O/cached.log
