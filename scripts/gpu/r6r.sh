# round 6: in-situ fused-core timing with the row-major V hand-off (d = 64 decode): GPU test, the
# driver command (check the QKV core at M ~ 480 is tgemm again) and B = 1-16 decode steps
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6r
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_tgemm_gpu.py -k "in_situ" > gpurun_out/r6r/tests.log 2>&1 || { tail -30 gpurun_out/r6r/tests.log; exit 1; }
tail -1 gpurun_out/r6r/tests.log
DLLM_GEMM_PLANS=gpurun_out/r6r/plans.json timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6r/bench.log 2>&1 || { tail -20 gpurun_out/r6r/bench.log; exit 1; }
grep '^{"metric"' gpurun_out/r6r/bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['p50_latency_ms'], d['init_s'], d['startup_s'])"
python3 -c "
import json; d=json.load(open('gpurun_out/r6r/plans.json'))
print({k: v for k, v in d.items() if k.startswith('c,') and int(k.split(',')[1]) in (448, 480, 512)})"
MB_DECODE_C=2048 MB_TEMP=0.8 MB_DECODE_B=1,2,4,8,16 DLLM_VERBOSE=1 timeout -k 10 500 python3 scripts/microbench.py --what decode > gpurun_out/r6r/tiny.log 2>&1 || { tail -20 gpurun_out/r6r/tiny.log; exit 1; }
grep '^{' gpurun_out/r6r/tiny.log | cut -c1-110
