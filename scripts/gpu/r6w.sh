# round 6: in-situ QKV timing against the engine's own KV pool: does QKV at the flagship's buckets
# pick the one-launch tgemm again, and the driver command (two arms)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6w
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_tgemm_gpu.py -k "in_situ" > gpurun_out/r6w/tests.log 2>&1 || { tail -20 gpurun_out/r6w/tests.log; exit 1; }
tail -1 gpurun_out/r6w/tests.log
for n in a b; do
  DLLM_GEMM_PLANS=gpurun_out/r6w/plans_$n.json timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6w/bench_$n.out 2>&1 || { tail -20 gpurun_out/r6w/bench_$n.out; exit 1; }
  grep '^{"metric"' gpurun_out/r6w/bench_$n.out | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['p50_latency_ms'], d['startup_s'])"
  python3 -c "
import json; d=json.load(open('gpurun_out/r6w/plans_$n.json'))
print({k: v for k, v in d.items() if k.startswith('c,') and ',2560,' in k and int(k.split(',')[1]) >= 192})"
done
