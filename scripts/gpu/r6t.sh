# round 6: driver command, fused cores timed in situ (a, c) vs the stand-in timings (b, d), same box
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6t
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
summ() {
  grep '^{"metric"' gpurun_out/r6t/bench_$1.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('$1', d['value'], d['p50_latency_ms'], d['init_s'], d.get('gpu_busy_sampled_pct'))"
}
arm() {
  local n=$1; shift
  timeout -k 10 500 python3 scripts/exp/bench_ab.py "$@" -- --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6t/bench_$n.log 2>&1 || { tail -20 gpurun_out/r6t/bench_$n.log; return 1; }
  summ $n
}
arm a && arm b gemm.FUSED_INSITU=0 && arm c && arm d gemm.FUSED_INSITU=0
