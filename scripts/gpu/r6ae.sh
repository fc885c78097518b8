# round 6 end-of-round check after the qkv_post change: full GPU suite, smoke, the driver bench command, profile
# then a kernel-level profile of the flagship (plans from the bench run, so no tuning in the trace)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6ae
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r6ae/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6ae/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6ae/smoke.log 2>&1 || { tail -20 gpurun_out/r6ae/smoke.log; exit 1; }
tail -1 gpurun_out/r6ae/smoke.log
DLLM_GEMM_PLANS=gpurun_out/r6ae/gemm_plans.json timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6ae/bench.out 2>&1 || { tail -20 gpurun_out/r6ae/bench.out; exit 1; }
grep '^{"metric"' gpurun_out/r6ae/bench.out > gpurun_out/r6ae/bench_line.json
python3 -c "
import json; d=json.load(open('gpurun_out/r6ae/bench_line.json')); print('bench', d['value'], d['p50_latency_ms'], d['startup_s'], d['kv_block_placement']['run_share'], d.get('gpu_busy_sampled_pct'))"
DLLM_GEMM_PLANS=gpurun_out/r6ae/gemm_plans.json timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r6ae/prof -o bench --output-format csv -- python3 bench.py --steps 6 --warmup 1 > gpurun_out/r6ae/prof_bench.out 2>&1 || { tail -20 gpurun_out/r6ae/prof_bench.out; exit 1; }
f=$(find gpurun_out/r6ae/prof -name "*kernel_stats.csv" | head -1)
python3 scripts/prof_summary.py "$f" 40 > gpurun_out/r6ae/kernels.md && head -12 gpurun_out/r6ae/kernels.md
find gpurun_out/r6ae/prof -name "*trace*" -delete
