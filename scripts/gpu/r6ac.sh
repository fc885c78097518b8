# round 6: qkv_post with dense units + V row-major hand-over: its tests, the driver's bench command,
# then the flagship kernel profile (plans from the bench run)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6ac
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_tgemm_gpu.py tests/test_kernels_gpu.py -m gpu -k "qkv_post or both_cores or in_situ or v_new or fused" > gpurun_out/r6ac/tests.log 2>&1 || { tail -30 gpurun_out/r6ac/tests.log; exit 1; }
tail -1 gpurun_out/r6ac/tests.log
DLLM_GEMM_PLANS=gpurun_out/r6ac/gemm_plans.json timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6ac/bench.out 2>&1 || { tail -20 gpurun_out/r6ac/bench.out; exit 1; }
grep '^{"metric"' gpurun_out/r6ac/bench.out > gpurun_out/r6ac/bench_line.json
python3 -c "
import json; d=json.load(open('gpurun_out/r6ac/bench_line.json')); print('bench', d['value'], d['p50_latency_ms'], d['startup_s'])"
python3 -c "
import json; d=json.load(open('gpurun_out/r6ac/gemm_plans.json'))
print('lin cores:', sorted(k for k, v in d.items() if k.startswith('c,') and v == 'lin'))"
DLLM_GEMM_PLANS=gpurun_out/r6ac/gemm_plans.json timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r6ac/prof -o bench --output-format csv -- python3 bench.py --steps 6 --warmup 1 > gpurun_out/r6ac/prof_bench.out 2>&1 || { tail -20 gpurun_out/r6ac/prof_bench.out; exit 1; }
f=$(find gpurun_out/r6ac/prof -name "*kernel_stats.csv" | head -1)
python3 scripts/prof_summary.py "$f" 40 > gpurun_out/r6ac/kernels.md && grep -i "qkv_post\|Cijk\|paged_attn" gpurun_out/r6ac/kernels.md
find gpurun_out/r6ac/prof -name "*trace*" -delete
