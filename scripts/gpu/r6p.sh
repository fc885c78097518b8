# round 6: fused-op cores timed through the fused ops (epilogue + row-scale prologue) at decode:
# TinyLlama / Llama-3-8B decode steps at B = 1-16, then the driver command, in-situ vs stand-in
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6p
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 MB_DECODE_C=2048 MB_TEMP=0.8
MB_DECODE_B=1,2,4,8,16 DLLM_VERBOSE=1 timeout -k 10 500 python3 scripts/microbench.py --what decode > gpurun_out/r6p/tiny.log 2>&1 || { tail -20 gpurun_out/r6p/tiny.log; exit 1; }
grep '^{' gpurun_out/r6p/tiny.log | cut -c1-120
MB_DECODE_B=1,2,4,8 DLLM_VERBOSE=1 timeout -k 10 600 python3 scripts/microbench.py --model llama-3-8b --what decode > gpurun_out/r6p/l8b.log 2>&1 || { tail -20 gpurun_out/r6p/l8b.log; exit 1; }
grep '^{' gpurun_out/r6p/l8b.log | cut -c1-120
summ() {
  grep '^{"metric"' gpurun_out/r6p/bench_$1.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('$1', d['value'], d['p50_latency_ms'], d['init_s'], d.get('gpu_busy_sampled_pct'))"
}
timeout -k 10 500 python3 scripts/exp/bench_ab.py -- --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6p/bench_a.log 2>&1 || { tail -20 gpurun_out/r6p/bench_a.log; exit 1; }
summ a
timeout -k 10 500 python3 scripts/exp/bench_ab.py gemm.FUSED_INSITU=0 -- --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6p/bench_b.log 2>&1 || { tail -20 gpurun_out/r6p/bench_b.log; exit 1; }
summ b
