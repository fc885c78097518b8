#!/bin/bash
# Early admission prefill (queued under a burst's last decode step) and the GIL switch interval:
# engine GPU tests, then the driver's bench window A/B on one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/ab13
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -k "engine or embedding or pipelin or burst" \
  -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { tail -30 $O/tests.log; exit $rc; }
export DLLM_GEMM_PLANS=$O/gemm_plans.json
i=0
for cfg in "1|5" "0|5" "1|0.5" "0|0.5" "1|5"; do
  i=$((i+1)); early=${cfg%|*}; gil=${cfg#*|}
  DLLM_EARLY_PREFILL=$early timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 --gil-switch-ms $gil > $O/run$i.log 2>&1 \
    || { echo "run $i failed"; tail -20 $O/run$i.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/run$i.log').read().strip().splitlines()[-1]); print('early=$early gil=$gil', d['value'], 'batch', d['avg_decode_batch'], 'p50', d['p50_latency_ms'], d['engine_time_split_s'])"
done
