#!/bin/bash
# In-burst joins (LLMEngine.BURST_JOIN): engine GPU tests, then the driver window A/B 1 / 0 / 1
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/ab18
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -4 $O/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/tests.log | head -30; exit $rc; }
export DLLM_GEMM_PLANS=$O/gemm_plans.json
i=0
for j in 1 0 1; do
  i=$((i+1))
  DLLM_BURST_JOIN=$j DLLM_SYNC_LOG=1 timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > $O/run$i.log 2>&1 \
    || { echo "run $i failed"; tail -30 $O/run$i.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/run$i.log').read().strip().splitlines()[-1]); print('join=$j', d['value'], 'batch', d['avg_decode_batch'], 'p50', d['p50_latency_ms'], 'ttft', d.get('ttft_ms_p50'), d.get('step_loop_sync'), d['engine_time_split_s'])"
done
