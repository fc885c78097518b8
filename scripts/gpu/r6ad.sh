# round 6: driver command, qkv_post V row-major hand-over on (a, c) vs off (b, d: V^T written by qkv_post), same box
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6ad
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
summ() {
  grep '^{"metric"' gpurun_out/r6ad/bench_$1.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('$1', d['value'], d['p50_latency_ms'], d['init_s'], d.get('gpu_busy_sampled_pct'))"
}
arm() {
  local n=$1; shift
  timeout -k 10 500 python3 scripts/exp/bench_ab.py "$@" -- --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6ad/bench_$n.log 2>&1 || { tail -20 gpurun_out/r6ad/bench_$n.log; return 1; }
  summ $n
}
arm a && arm b gemm.QKV_POST_VROWS=0 && arm c && arm d gemm.QKV_POST_VROWS=0
