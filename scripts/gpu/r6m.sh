# round 6: prefill GEMM core A/B on the driver command: hipBLASLt + standalone epilogues (default)
# vs the tuned prefill buckets (gemm.PREFILL_TUNE=1) whose candidates now include the grouped-raster
# and 8-loader 256 x 128 tgemm plans; same box, same decode plans (a, c: off; b: on)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6m
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
summ() {
  grep '^{"metric"' gpurun_out/r6m/bench_$1.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('$1', d['value'], d['p50_latency_ms'], d['engine_time_split_s']['step_loop']['t_prefill_s'], d.get('gpu_busy_sampled_pct'))"
}
DLLM_GEMM_PLANS=gpurun_out/r6m/plans_off.json timeout -k 10 400 python3 scripts/exp/bench_ab.py -- --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6m/bench_a.log 2>&1 || { tail -20 gpurun_out/r6m/bench_a.log; exit 1; }
summ a
cp gpurun_out/r6m/plans_off.json gpurun_out/r6m/plans_on.json
DLLM_VERBOSE=1 DLLM_GEMM_PLANS=gpurun_out/r6m/plans_on.json timeout -k 10 500 python3 scripts/exp/bench_ab.py gemm.PREFILL_TUNE=1 -- --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6m/bench_b.log 2>&1 || { tail -20 gpurun_out/r6m/bench_b.log; exit 1; }
summ b
grep "gemm prefill" gpurun_out/r6m/bench_b.log | cut -c1-200
DLLM_GEMM_PLANS=gpurun_out/r6m/plans_off.json timeout -k 10 400 python3 scripts/exp/bench_ab.py -- --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6m/bench_c.log 2>&1 || { tail -20 gpurun_out/r6m/bench_c.log; exit 1; }
summ c
