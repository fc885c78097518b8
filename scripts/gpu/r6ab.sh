# round 6: driver command, split-form margin 1.03 (a, c; default) vs 1.15 (b, d: a one-launch fused
# core unless hipBLASLt + standalone epilogue is > 15 % faster), same box; fused-core choices printed
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6ab
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
arm() {
  local n=$1; shift
  DLLM_GEMM_PLANS=gpurun_out/r6ab/plans_$n.json timeout -k 10 500 python3 scripts/exp/bench_ab.py "$@" -- --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6ab/bench_$n.log 2>&1 || { tail -20 gpurun_out/r6ab/bench_$n.log; return 1; }
  grep '^{"metric"' gpurun_out/r6ab/bench_$n.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['p50_latency_ms'], d['startup_s'])"
  python3 -c "
import json; d=json.load(open('gpurun_out/r6ab/plans_$n.json'))
print('$n lin cores:', sorted(k for k, v in d.items() if k.startswith('c,') and v == 'lin'))"
}
arm a && arm b gemm.SPLIT_MARGIN=1.15 && arm c && arm d gemm.SPLIT_MARGIN=1.15
