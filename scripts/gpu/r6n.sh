# round 6: the new defaults on the driver command, same box: prefill core autotuned (tgemm where it
# wins) vs hipBLASLt prefill (gemm.PREFILL_TUNE=0); KV runs start mid-stretch after a live tail.
# Order: off, on, on, off (on-arms share one plan file with the prefill entries; off-arms one without)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6n
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
summ() {
  grep '^{"metric"' gpurun_out/r6n/bench_$1.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); k=d['kv_block_placement']
print('$1', d['value'], d['p50_latency_ms'], d['engine_time_split_s']['step_loop']['t_prefill_s'], d.get('gpu_busy_sampled_pct'), d['prefix_cache_hit_rate'], k['run_share'], k['run_miss_held_share'], k['roomy_stretch_mean_blocks'])"
}
arm() {  # name, plans file, overrides...
  local n=$1 p=$2; shift 2
  DLLM_GEMM_PLANS=gpurun_out/r6n/$p timeout -k 10 500 python3 scripts/exp/bench_ab.py "$@" -- --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6n/bench_$n.log 2>&1 || { tail -20 gpurun_out/r6n/bench_$n.log; return 1; }
  summ $n
}
arm b plans_off.json gemm.PREFILL_TUNE=0 && cp gpurun_out/r6n/plans_off.json gpurun_out/r6n/plans_on.json && \
arm a plans_on.json && arm c plans_on.json && arm d plans_off.json gemm.PREFILL_TUNE=0
