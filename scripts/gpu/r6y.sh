# round 6: decode attention persistent grid A/B on the driver command (same box, shared GEMM plans)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6y
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 DLLM_GEMM_PLANS=gpurun_out/r6y/plans.json
arm() {
  local n=$1; shift
  timeout -k 10 500 python3 scripts/exp/bench_ab.py "$@" -- --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6y/bench_$n.log 2>&1 || { tail -20 gpurun_out/r6y/bench_$n.log; return 1; }
  grep '^{"metric"' gpurun_out/r6y/bench_$n.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['p50_latency_ms'], d['engine_time_split_s']['step_loop']['t_decode_gpu_wait_s'])"
}
arm a && arm b engine.ATTN_PGRID=1024 && arm c engine.ATTN_PGRID=768 && arm d
