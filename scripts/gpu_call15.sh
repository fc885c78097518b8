#!/bin/bash
# Decode-step I/O kernels (ops.step_fetch / step_store inside the step graph): numerics, engine GPU
# tests, then the driver's window with DLLM_STEP_IO_KERNEL 1 / 0 / 1
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/ab15
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "step_fetch or embedding or engine or pipelin or burst or graph" \
  -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { tail -40 $O/tests.log; exit $rc; }
export DLLM_GEMM_PLANS=$O/gemm_plans.json
i=0
for gio in 1 0 1; do
  i=$((i+1))
  DLLM_STEP_IO_KERNEL=$gio timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > $O/run$i.log 2>&1 \
    || { echo "run $i failed"; tail -20 $O/run$i.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/run$i.log').read().strip().splitlines()[-1]); print('gio=$gio', d['value'], 'batch', d['avg_decode_batch'], 'p50', d['p50_latency_ms'], d['engine_time_split_s'])"
done
