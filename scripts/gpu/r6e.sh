# round 6: driver-command A/B of the KV placement (round-6 default vs round-5 runs), same box,
# one GEMM plan file for all arms; then the whole GPU test suite
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6e
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 DLLM_GEMM_PLANS=gpurun_out/r6e/plans.json
for arm in "a engine.KV_PLACEMENT=2" "b engine.KV_PLACEMENT=1" "c engine.KV_PLACEMENT=2"; do
  set -- $arm
  timeout -k 10 400 python3 scripts/exp/bench_ab.py $2 -- --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6e/bench_$1.log 2>&1 || { tail -20 gpurun_out/r6e/bench_$1.log; exit 1; }
  grep '^{' gpurun_out/r6e/bench_$1.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('$1', '$2', d['value'], d['p50_latency_ms'], d['prefix_cache_hit_rate'], d['kv_block_placement'], d.get('gpu_busy_sampled_pct'), d['avg_decode_batch'])"
done
timeout -k 10 1100 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r6e/gpu_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r6e/gpu_tests.log
exit $rc
